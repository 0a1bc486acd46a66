// gpr/SparseGaussianProcess.h — SparseGaussianProcess<T> (subset of regressors) over libgprx.
//
// Same public surface as the reference (include/SparseGaussianProcess.h:30-141):
// AddInducingSample, ClearInducingSamples, Predict, operator()(x,y),
// GetNumberOfInducingSamples, Get/SetJitter, Initialize.  Initialize is one
// gprx_sparse_fit call (Knm streamed through the GPU in row blocks, never materialised in
// full; the N x N core matrix of :309-311 is not formed).  Predict runs on the device
// through a resident model holding the inducing points and the regression vectors.
#pragma once

#include <string>
#include <vector>

#include "GaussianProcess.h"

namespace gpr {

template <class TScalarType>
class SparseGaussianProcess : public GaussianProcess<TScalarType> {
public:
    typedef SparseGaussianProcess Self;
    typedef std::shared_ptr<Self> Pointer;
    typedef GaussianProcess<TScalarType> Superclass;
    typedef typename Superclass::VectorType VectorType;
    typedef typename Superclass::MatrixType MatrixType;
    typedef typename Superclass::VectorListType VectorListType;
    typedef typename Superclass::KernelTypePointer KernelTypePointer;

    explicit SparseGaussianProcess(KernelTypePointer kernel) : Superclass(kernel), m_Jitter(0) {}
    SparseGaussianProcess(KernelTypePointer kernel, TScalarType jitter) : Superclass(kernel), m_Jitter(jitter) {}
    ~SparseGaussianProcess() override {
        if (m_Sparse) gprx_model_destroy(m_Sparse);
    }

    // include/SparseGaussianProcess.h:61-75
    void AddInducingSample(const VectorType& x, const VectorType& y) {
        if (m_InducingSampleVectors.empty()) this->m_InputDimension = (unsigned)x.size();
        if (m_InducingLabelVectors.empty()) this->m_OutputDimension = (unsigned)y.size();
        this->CheckInputDimension(x, "SparseGaussianProcess::AddInducingSample: ");
        this->CheckOutputDimension(y, "SparseGaussianProcess::AddInducingSample: ");
        m_InducingSampleVectors.push_back(x);
        m_InducingLabelVectors.push_back(y);
        m_SparseInitialized = false;
    }
    void ClearInducingSamples() {
        m_InducingSampleVectors.clear();
        m_InducingLabelVectors.clear();
        m_SparseInitialized = false;
    }
    unsigned GetNumberOfInducingSamples() const { return (unsigned)m_InducingSampleVectors.size(); }
    TScalarType GetJitter() const { return m_Jitter; }
    void SetJitter(TScalarType jitter) {
        m_Jitter = jitter;
        m_SparseInitialized = false;
    }

    // include/SparseGaussianProcess.h:86-92: Kx^T RV over the inducing points
    VectorType Predict(const VectorType& x) override {
        Initialize();
        this->CheckInputDimension(x, "GaussianProcess::Predict: ");
        VectorType mean(this->m_OutputDimension);
        ThrowIfFailed(gprx_model_predict(m_Sparse, x.data(), 1, mean.data(), nullptr), DefaultContext());
        return mean;
    }

    // include/SparseGaussianProcess.h:94-106: k(x,y) - Kx^T Kinv Ky + Kx^T RM Ky, on the
    // device against the resident W = Kinv - RM (gprx_model_set_sparse_cov)
    TScalarType operator()(const VectorType& x, const VectorType& y) override {
        Initialize();
        this->CheckInputDimension(x, "SparseGaussianProcess::(): ");
        this->CheckInputDimension(y, "SparseGaussianProcess::(): ");
        TScalarType out = 0;
        ThrowIfFailed(gprx_model_posterior_cov(m_Sparse, x.data(), y.data(), 1, &out), DefaultContext());
        return out;
    }

    // include/SparseGaussianProcess.h:108-128
    void Initialize() override {
        if (m_SparseInitialized) return;
        if (m_InducingSampleVectors.empty())
            throw std::string("SparseGaussianProcess::Initialize: no inducing samples defined during initialization");
        if (m_InducingLabelVectors.empty())
            throw std::string("SparseGaussianProcess::Initialize: no inducing labels defined during initialization");
        if (this->m_SampleVectors.empty())
            throw std::string("SparseGaussianProcess::Initialize: no dense samples defined during initialization");
        if (this->m_LabelVectors.empty())
            throw std::string("SparseGaussianProcess::Initialize: no dense labels defined during initialization");
        const std::size_t M = m_InducingSampleVectors.size(), n = this->m_SampleVectors.size();
        if (!(M <= n))
            throw std::string(
                "SparseGaussianProcess::ComputeKernelVectorMatrix: number of dense samples must be higher than the "
                "number of sparse samples");
        const unsigned d = this->m_InputDimension, m = this->m_OutputDimension;
        std::vector<TScalarType> X = Pack(this->m_SampleVectors), Y = Pack(this->m_LabelVectors),
                                 Xm = Pack(m_InducingSampleVectors), Ym = Pack(m_InducingLabelVectors);
        m_Kinv.assign(M * M, 0);
        m_RM.assign(M * M, 0);
        m_RegressionVectors.resize(M, m);
        gprx_kernel_desc kd = Desc();
        ThrowIfFailed(gprx_sparse_fit(DefaultContext(), Dtype(), &kd, X.data(), Y.data(), (int64_t)n, (int32_t)d,
                                      (int32_t)m, Xm.data(), (int64_t)M, (double)this->m_Sigma, (double)m_Jitter,
                                      m_Kinv.data(), m_RegressionVectors.data(), m_RM.data()),
                      DefaultContext());
        if (!m_Sparse) ThrowIfFailed(gprx_model_create(DefaultContext(), Dtype(), &m_Sparse), DefaultContext());
        ThrowIfFailed(gprx_model_set_data(m_Sparse, Xm.data(), Ym.data(), (int64_t)M, (int32_t)d, (int32_t)m),
                      DefaultContext());
        ThrowIfFailed(gprx_model_set_kernel(m_Sparse, &kd), DefaultContext());
        ThrowIfFailed(gprx_model_set_alpha(m_Sparse, m_RegressionVectors.data()), DefaultContext());
        std::vector<TScalarType> W(M * M);
        for (std::size_t i = 0; i < M * M; i++) W[i] = m_Kinv[i] - m_RM[i];
        ThrowIfFailed(gprx_model_set_sparse_cov(m_Sparse, W.data()), DefaultContext());
        m_SparseInitialized = true;
    }

    // SparseGaussianLogLikelihood (include/SparseLikelihood.h:231-344) on the device: one
    // gprx_sparse_lml call over the current dense and inducing samples (SparseLikelihood.h in
    // this directory is the reference's class surface over it).  grad receives the kernel
    // parameters' derivatives (GetParameters order).
    void EvaluateLogLikelihood(bool want_grad, bool compat, double* value, std::vector<double>* grad,
                               double* logdet) const {
        if (m_InducingSampleVectors.empty())
            throw std::string("SparseLikelihood::GetValueAndParameterDerivative: there are no inducing samples specified");
        if (this->m_SampleVectors.empty())
            throw std::string("SparseGaussianProcess::ComputeCoreMatrices: empty sample set.");
        const std::size_t M = m_InducingSampleVectors.size(), n = this->m_SampleVectors.size();
        if (!(M <= n))
            throw std::string(
                "SparseGaussianProcess::ComputeKernelVectorMatrix: number of dense samples must be higher than the "
                "number of sparse samples");
        if (this->m_OutputDimension != 1)
            throw std::string("SparseGaussianLogLikelihood: device likelihood supports one output dimension");
        const unsigned d = this->m_InputDimension;
        std::vector<TScalarType> X = Pack(this->m_SampleVectors), Y = Pack(this->m_LabelVectors),
                                 Xm = Pack(m_InducingSampleVectors);
        gprx_kernel_desc kd = Desc();
        std::vector<double> g(3 * GPRX_MAX_KNODES, 0.0);
        int32_t np = 0;
        const uint32_t flags = (want_grad ? GPRX_LML_GRAD : 0u) | (compat ? GPRX_LML_COMPAT : 0u);
        ThrowIfFailed(gprx_sparse_lml(DefaultContext(), Dtype(), &kd, X.data(), Y.data(), (int64_t)n, (int32_t)d, 1,
                                      Xm.data(), (int64_t)M, (double)this->m_Sigma, (double)m_Jitter, flags, value,
                                      want_grad ? g.data() : nullptr, &np, logdet),
                      DefaultContext());
        if (grad) grad->assign(g.begin(), g.begin() + np);
    }

    const MatrixType& GetRegressionVectors() const { return m_RegressionVectors; }
    const std::vector<TScalarType>& GetInducingInvertedKernelMatrix() const { return m_Kinv; }  // row-major M x M
    const std::vector<TScalarType>& GetRegressionMatrix() const { return m_RM; }               // row-major M x M

private:
    static gprx_dtype Dtype() { return sizeof(TScalarType) == 8 ? GPRX_F64 : GPRX_F32; }
    gprx_kernel_desc Desc() const {
        std::vector<gprx_knode> prog;
        this->m_Kernel->Describe(prog);
        if (prog.size() > GPRX_MAX_KNODES) throw std::string("SparseGaussianProcess: kernel has too many nodes");
        gprx_kernel_desc kd{};
        kd.n_nodes = (int32_t)prog.size();
        for (std::size_t i = 0; i < prog.size(); i++) kd.node[i] = prog[i];
        return kd;
    }
    static std::vector<TScalarType> Pack(const VectorListType& v) {
        std::vector<TScalarType> out;
        for (const auto& x : v)
            for (std::size_t k = 0; k < x.size(); k++) out.push_back(x[k]);
        return out;
    }

    TScalarType m_Jitter;
    bool m_SparseInitialized = false;
    VectorListType m_InducingSampleVectors;
    VectorListType m_InducingLabelVectors;
    MatrixType m_RegressionVectors;
    std::vector<TScalarType> m_Kinv, m_RM;
    gprx_model* m_Sparse = nullptr;
};

}  // namespace gpr
