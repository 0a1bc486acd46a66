// gpr/GaussianProcess.h — GaussianProcess<T> host API over libgprx.
//
// Same public surface as the reference class (include/GaussianProcess.h:33-328):
// AddSample, Initialize, Predict, PredictDerivative, operator()(x,y), GetCredibleInterval,
// Get/SetKernel, Get/SetSigma, SetInversionMethod, Get/SetEfficientStorage, Save, Load,
// ToString, Lock/UnLock, operator==.  The numerics are done by libgprx on the GPU: the
// training set, the Cholesky factor of K + sigma^2 I and the regression vectors stay
// resident in HBM; the host keeps the sample lists (for Save / ==) and a copy of the
// regression vectors (m_RegressionVectors, as the reference).
//
// Kernels with no device form (a user Kernel<T> subclass that does not override Describe):
// K, the query kernel vectors and the derivative matrices are evaluated on the host through
// the virtual operator() / GetDerivative, as the reference does for every kernel; the
// factorisation, solves and reductions still run on the device (gprx_model_set_kernel_matrix
// and the *_kx entry points of include/gprx.h).
//
// Differences (documented in DESIGN.md): the core matrix C = (K + sigma^2 I)^{-1} is
// materialised lazily from the device factor (Save, GetCoreMatrix), not at every
// Initialize; operator()/GetCredibleInterval use the factor (k - |L^{-1}k|^2) instead of
// Kx^T C Ky.  InversionMethod (lib/GaussianProcess.cpp:531-618): FullPivotLU (default) and
// SelfAdjointEigenSolver factorise with Cholesky and, when K + sigma^2 I is not numerically
// positive definite, fall back to a partial-pivot LU in double (FullPivotLU = dgetrf_,
// include/LAPACKUtils.h:38-56; gpr_amd/csrc/k_getrf.hip); JacobiSVD / BDCSVD, whose formula is
// the exact inverse V S^{-1} U^T, factorise with that LU directly (no SVD is formed).
//
// Threading (reference: tests/PosteriorProcessTest.cpp:120-134 calls Predict and operator()
// concurrently after Initialize): the read-only calls may run concurrently; the lazy device
// refit behind operator()/GetCoreMatrix after Load is guarded by m_DevMu, and libgprx
// serialises the device calls of one context.
#pragma once

#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../gprx.h"
#include "Kernel.h"
#include "Matrix.h"

namespace gpr {

template <class T>
class Likelihood;
template <class T>
class GaussianLogLikelihood;
template <class T>
class GaussianLikelihood;

// Process-wide libgprx context (device from $GPRX_DEVICE, default 0).  Throws std::string
// when no GPU is visible: there is no CPU fallback.
gprx_ctx* DefaultContext();
// Throw the reference-style std::string for a failed libgprx call.
void ThrowIfFailed(gprx_status st, gprx_ctx* ctx);

template <class TScalarType>
class GaussianProcess {
public:
    typedef GaussianProcess Self;
    typedef std::shared_ptr<Self> Pointer;
    typedef Kernel<TScalarType> KernelType;
    typedef typename KernelType::Pointer KernelTypePointer;
    typedef DenseVector<TScalarType> VectorType;
    typedef DenseMatrix<TScalarType> MatrixType;
    typedef std::vector<VectorType> VectorListType;
    typedef long double HighPrecisionType;
    typedef enum { FullPivotLU = 0, JacobiSVD = 1, BDCSVD = 2, SelfAdjointEigenSolver = 3 } InversionMethod;

    explicit GaussianProcess(KernelTypePointer kernel);
    virtual ~GaussianProcess();
    GaussianProcess(const Self&) = delete;
    void operator=(const Self&) = delete;

    void AddSample(const VectorType& x, const VectorType& y);
    virtual VectorType Predict(const VectorType& x);
    virtual VectorType PredictDerivative(const VectorType& x, MatrixType& D);
    virtual TScalarType operator()(const VectorType& x, const VectorType& y);
    TScalarType GetCredibleInterval(const VectorType& x);
    virtual void Initialize();

    // Batched, device-native forms (one launch for all rows; not in the reference).
    MatrixType PredictBatch(const MatrixType& Xq);                 // rows = queries -> q x m
    std::vector<TScalarType> CredibleIntervalBatch(const MatrixType& Xq);

    const KernelTypePointer GetKernel() { return m_Kernel; }
    void SetKernel(KernelTypePointer k) {
        m_Kernel = k;
        m_Initialized = false;
    }
    void DebugOn() { debug = true; }
    virtual unsigned GetNumberOfSamples() const { return (unsigned)m_SampleVectors.size(); }
    TScalarType GetSigma() const { return m_Sigma; }
    TScalarType GetSigmaSquared() const { return m_Sigma * m_Sigma; }
    void SetSigma(TScalarType sigma) {
        m_Sigma = sigma;
        m_Initialized = false;
    }
    virtual unsigned GetNumberOfInputDimensions() const { return m_InputDimension; }
    virtual void SetInversionMethod(InversionMethod m) { m_InvMethod = m; }
    virtual InversionMethod GetInversionMethod() { return m_InvMethod; }
    bool GetEfficientStorage() { return m_EfficientStorage; }
    void SetEfficientStorage(bool s) { m_EfficientStorage = s; }

    virtual void Save(std::string prefix);
    virtual void Load(std::string prefix);
    virtual void ToString() const;

    void Lock() { gp_lock.lock(); }
    void UnLock() { gp_lock.unlock(); }

    virtual bool operator==(const GaussianProcess<TScalarType>& b) const;
    virtual bool operator!=(const GaussianProcess<TScalarType>& b) const { return !operator==(b); }

    // The explicit core matrix (K + sigma^2 I)^{-1}, materialised from the device factor.
    const MatrixType& GetCoreMatrix();

protected:
    KernelTypePointer m_Kernel;
    TScalarType m_Sigma;
    VectorListType m_SampleVectors;
    VectorListType m_LabelVectors;
    MatrixType m_RegressionVectors;
    MatrixType m_CoreMatrix;
    bool m_Initialized;
    unsigned m_InputDimension;
    unsigned m_OutputDimension;
    InversionMethod m_InvMethod;
    bool m_EfficientStorage;
    std::mutex gp_lock;
    bool debug;

    gprx_model* m_Model = nullptr;
    std::mutex m_DevMu;           // guards the lazy refit (EnsureFactor), m_CoreMatrix/m_CoreSize
    bool m_DeviceFactor = false;  // device holds the Cholesky factor of the current state
    bool m_HostKernel = false;    // the kernel has no device form (Describe throws): K and the
                                  // kernel vectors are evaluated here through the virtual
                                  // operator() (include/Kernel.h:52-59), the rest on the device
    bool m_CoreValid = false;     // m_CoreMatrix holds the materialised core matrix
    bool m_DataUploaded = false;  // the device model holds the current samples (AddSample clears
                                  // it): an optimiser loop re-evaluating the likelihood under new
                                  // kernel parameters re-sends only the kernel
    std::size_t m_CoreSize = 0;   // the reference's m_CoreMatrix.diagonalSize(): n once the
                                  // core exists (Initialize w/o efficient storage, operator(),
                                  // Load), 0 when efficient storage dropped it

    void CheckInputDimension(const VectorType& x, std::string msg_prefix) const;
    void CheckOutputDimension(const VectorType& y, std::string msg_prefix) const;
    gprx_model* Model();
    void UploadState();            // samples, kernel, noise -> device
    void FitDevice(gprx_fit_info* info = nullptr);
    void EnsureFactor();           // factor for operator()/core; keeps the regression vectors
                                   // (caller holds m_DevMu)
    // host-evaluated kernel rows K(x, X) of q queries (rows of Xq, or one vector), row-major
    std::vector<TScalarType> HostKernelRows(const TScalarType* Xq, std::size_t q) const;
    std::vector<TScalarType> HostDerivativeMatrices(int32_t& P) const;  // P x n x n

    friend class Likelihood<TScalarType>;
};

}  // namespace gpr
