// GaussianProcess.cpp — host implementation of gpr::GaussianProcess<T> over libgprx.
//
// Call structure mirrors the reference (lib/GaussianProcess.cpp): Initialize ->
// ComputeRegressionVectors, with the covariance build, factorisation and solve moved to
// one device call (gprx_model_fit); Predict/PredictDerivative/operator() call the batched
// device kernels with q = 1.  Error messages are the reference's std::string messages.
#include "../../include/gpr/GaussianProcess.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <limits>
#include <sstream>
#include <sys/stat.h>
#include <thread>

#include "../../include/gpr/MatrixIO.h"

namespace gpr {

void ThrowIfFailed(gprx_status st, gprx_ctx* ctx) {
    if (st == GPRX_OK) return;
    throw std::string(gprx_last_error(ctx));
}

gprx_ctx* DefaultContext() {
    static std::mutex mu;
    static gprx_ctx* ctx = nullptr;
    std::lock_guard<std::mutex> lk(mu);
    if (!ctx) {
        int dev = 0;
        if (const char* e = std::getenv("GPRX_DEVICE")) dev = std::atoi(e);
        gprx_status st = gprx_ctx_create(dev, &ctx);
        if (st != GPRX_OK) {
            ctx = nullptr;
            throw std::string(gprx_last_error(nullptr));
        }
    }
    return ctx;
}

template <class T>
static gprx_dtype dtype_of();
template <>
gprx_dtype dtype_of<double>() {
    return GPRX_F64;
}
template <>
gprx_dtype dtype_of<float>() {
    return GPRX_F32;
}

static bool file_ok(const std::string& f) {
    struct stat st;
    return stat(f.c_str(), &st) == 0 && !S_ISDIR(st.st_mode);
}

template <class T>
GaussianProcess<T>::GaussianProcess(KernelTypePointer kernel)
    : m_Kernel(kernel),
      m_Sigma(0),
      m_Initialized(false),
      m_InputDimension(0),
      m_OutputDimension(0),
      m_InvMethod(FullPivotLU),
      m_EfficientStorage(false),
      debug(false) {}

template <class T>
GaussianProcess<T>::~GaussianProcess() {
    if (m_Model) gprx_model_destroy(m_Model);
}

template <class T>
gprx_model* GaussianProcess<T>::Model() {
    if (!m_Model) ThrowIfFailed(gprx_model_create(DefaultContext(), dtype_of<T>(), &m_Model), DefaultContext());
    return m_Model;
}

// lib/GaussianProcess.cpp:36-51
template <class T>
void GaussianProcess<T>::AddSample(const VectorType& x, const VectorType& y) {
    if (m_SampleVectors.empty()) m_InputDimension = (unsigned)x.size();
    if (m_LabelVectors.empty()) m_OutputDimension = (unsigned)y.size();
    CheckInputDimension(x, "GaussianProcess::AddSample: ");
    CheckOutputDimension(y, "GaussianProcess::AddSample: ");
    m_SampleVectors.push_back(x);
    m_LabelVectors.push_back(y);
    m_Initialized = false;
    m_DataUploaded = false;
}

template <class T>
void GaussianProcess<T>::UploadState() {
    gprx_ctx* ctx = DefaultContext();
    const std::size_t n = m_SampleVectors.size();
    if (!m_DataUploaded || !m_Model) {
        const std::size_t d = m_InputDimension, m = m_OutputDimension;
        std::vector<T> X(n * d), Y(n * m);
        for (std::size_t i = 0; i < n; i++) {
            for (std::size_t k = 0; k < d; k++) X[i * d + k] = m_SampleVectors[i][k];
            for (std::size_t c = 0; c < m; c++) Y[i * m + c] = m_LabelVectors[i][c];
        }
        ThrowIfFailed(gprx_model_set_data(Model(), X.data(), Y.data(), (int64_t)n, (int32_t)d, (int32_t)m), ctx);
        m_DataUploaded = true;
    }
    std::vector<gprx_knode> prog;
    try {
        m_Kernel->Describe(prog);
        m_HostKernel = false;
    } catch (const std::string&) {
        // no device form: K through the virtual operator() (lib/GaussianProcess.cpp:384-402),
        // the upper triangle mirrored, evaluated over the rows by the host's threads
        m_HostKernel = true;
        std::vector<T> K(n * n);
        const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        std::vector<std::thread> th;
        std::exception_ptr err = nullptr;
        std::mutex emu;
        for (unsigned w = 0; w < nt; w++)
            th.emplace_back([&, w]() {
                try {
                    for (std::size_t i = w; i < n; i += nt)
                        for (std::size_t j = 0; j <= i; j++)
                            K[i * n + j] = K[j * n + i] = (*m_Kernel)(m_SampleVectors[i], m_SampleVectors[j]);
                } catch (...) {
                    std::lock_guard<std::mutex> l(emu);
                    if (!err) err = std::current_exception();
                }
            });
        for (auto& t : th) t.join();
        if (err) std::rethrow_exception(err);
        ThrowIfFailed(gprx_model_set_kernel_matrix(m_Model, K.data()), ctx);
        ThrowIfFailed(gprx_model_set_noise(m_Model, (double)m_Sigma), ctx);
        return;
    }
    if (prog.size() > GPRX_MAX_KNODES) throw std::string("GaussianProcess: kernel has too many nodes for the device");
    gprx_kernel_desc desc{};
    desc.n_nodes = (int32_t)prog.size();
    for (std::size_t i = 0; i < prog.size(); i++) desc.node[i] = prog[i];
    ThrowIfFailed(gprx_model_set_kernel(m_Model, &desc), ctx);
    ThrowIfFailed(gprx_model_set_noise(m_Model, (double)m_Sigma), ctx);
}

template <class T>
void GaussianProcess<T>::FitDevice(gprx_fit_info* info) {
    UploadState();
    gprx_fit_info fi;
    // lib/GaussianProcess.cpp:531-618: FullPivotLU (default) and SelfAdjointEigenSolver take
    // the Cholesky with the LU fallback; the SVD methods (the exact inverse V S^-1 U^T) take
    // the LU in double directly (include/gprx.h GPRX_FIT_FORCE_LU)
    const uint32_t flags = (m_InvMethod == JacobiSVD || m_InvMethod == BDCSVD) ? GPRX_FIT_FORCE_LU : GPRX_FIT_DEFAULT;
    ThrowIfFailed(gprx_model_fit(m_Model, flags, &fi), DefaultContext());
    if (info) *info = fi;
    m_DeviceFactor = true;
}

// The factor for operator()/core matrix.  A GP whose regression vectors are fixed (loaded
// by Load, or computed by Initialize) keeps predicting with them, as the reference does:
// the refit's alpha is replaced by m_RegressionVectors.
template <class T>
void GaussianProcess<T>::EnsureFactor() {  // m_DevMu held
    if (m_DeviceFactor) return;
    FitDevice();
    if (m_Initialized && m_RegressionVectors.rows() == m_SampleVectors.size())
        ThrowIfFailed(gprx_model_set_alpha(m_Model, m_RegressionVectors.data()), DefaultContext());
}

template <class T>
std::vector<T> GaussianProcess<T>::HostKernelRows(const T* Xq, std::size_t q) const {
    const std::size_t n = m_SampleVectors.size(), d = m_InputDimension;
    std::vector<T> R(q * n);
    VectorType x(d);
    for (std::size_t a = 0; a < q; a++) {
        for (std::size_t k = 0; k < d; k++) x[k] = Xq[a * d + k];
        for (std::size_t i = 0; i < n; i++) R[a * n + i] = (*m_Kernel)(x, m_SampleVectors[i]);
    }
    return R;
}

// dK/dp for every parameter p (GetDerivative order), P x n x n
template <class T>
std::vector<T> GaussianProcess<T>::HostDerivativeMatrices(int32_t& P) const {
    const std::size_t n = m_SampleVectors.size();
    P = (int32_t)m_Kernel->GetNumberOfParameters();
    std::vector<T> D((std::size_t)P * n * n);
    for (std::size_t i = 0; i < n; i++)
        for (std::size_t j = 0; j <= i; j++) {
            const VectorType g = m_Kernel->GetDerivative(m_SampleVectors[i], m_SampleVectors[j]);
            if ((int32_t)g.size() != P) throw std::string("GaussianProcess: kernel derivative has the wrong size");
            for (int32_t p = 0; p < P; p++) D[(std::size_t)p * n * n + i * n + j] = D[(std::size_t)p * n * n + j * n + i] = g[p];
        }
    return D;
}

// lib/GaussianProcess.cpp:118-130, 642-672
template <class T>
void GaussianProcess<T>::Initialize() {
    if (m_Initialized) return;
    if (!(m_SampleVectors.size() > 0))
        throw std::string("GaussianProcess::Initialize: no input samples defined during initialization");
    if (!(m_LabelVectors.size() > 0))
        throw std::string("GaussianProcess::Initialize: no ouput labels defined during initialization");
    if (debug) std::cout << "GaussianProcess::ComputeRegressionVectors: calculating regression vectors... " << std::endl;
    FitDevice();
    m_RegressionVectors.resize(m_SampleVectors.size(), m_OutputDimension);
    ThrowIfFailed(gprx_model_get_alpha(m_Model, m_RegressionVectors.data()), DefaultContext());
    m_CoreValid = false;
    m_CoreMatrix.resize(0, 0);
    // lib/GaussianProcess.cpp:652-668: the core exists unless efficient storage drops it
    m_CoreSize = m_EfficientStorage ? 0 : m_SampleVectors.size();
    m_Initialized = true;
}

template <class T>
const typename GaussianProcess<T>::MatrixType& GaussianProcess<T>::GetCoreMatrix() {
    Initialize();
    std::lock_guard<std::mutex> lk(m_DevMu);
    if (!m_CoreValid) {
        EnsureFactor();
        const std::size_t n = m_SampleVectors.size();
        m_CoreMatrix.resize(n, n);
        ThrowIfFailed(gprx_model_core_matrix(m_Model, m_CoreMatrix.data()), DefaultContext());
        m_CoreValid = true;
    }
    m_CoreSize = m_SampleVectors.size();
    return m_CoreMatrix;
}

// lib/GaussianProcess.cpp:54-61
template <class T>
typename GaussianProcess<T>::VectorType GaussianProcess<T>::Predict(const VectorType& x) {
    Initialize();
    CheckInputDimension(x, "GaussianProcess::Predict: ");
    VectorType mean(m_OutputDimension);
    std::lock_guard<std::mutex> lk(m_DevMu);  // not inside another thread's lazy refit
    if (m_HostKernel) {
        const std::vector<T> kx = HostKernelRows(x.data(), 1);
        ThrowIfFailed(gprx_model_predict_kx(m_Model, kx.data(), x.data(), 1, mean.data(), nullptr), DefaultContext());
        return mean;
    }
    ThrowIfFailed(gprx_model_predict(m_Model, x.data(), 1, mean.data(), nullptr), DefaultContext());
    return mean;
}

template <class T>
typename GaussianProcess<T>::MatrixType GaussianProcess<T>::PredictBatch(const MatrixType& Xq) {
    Initialize();
    if (Xq.cols() != m_InputDimension) throw std::string("GaussianProcess::PredictBatch: dimension mismatch");
    MatrixType out(Xq.rows(), m_OutputDimension);
    std::lock_guard<std::mutex> lk(m_DevMu);
    if (m_HostKernel) {
        const std::vector<T> kx = HostKernelRows(Xq.data(), Xq.rows());
        ThrowIfFailed(gprx_model_predict_kx(m_Model, kx.data(), Xq.data(), (int64_t)Xq.rows(), out.data(), nullptr),
                      DefaultContext());
        return out;
    }
    ThrowIfFailed(gprx_model_predict(m_Model, Xq.data(), (int64_t)Xq.rows(), out.data(), nullptr), DefaultContext());
    return out;
}

// lib/GaussianProcess.cpp:64-81: D is d x m, D(:,c) = -X^T (Kx o alpha_c)
template <class T>
typename GaussianProcess<T>::VectorType GaussianProcess<T>::PredictDerivative(const VectorType& x, MatrixType& D) {
    Initialize();
    CheckInputDimension(x, "GaussianProcess::PredictDerivative: ");
    VectorType mean(m_OutputDimension);
    D.resize(m_InputDimension, m_OutputDimension);
    std::lock_guard<std::mutex> lk(m_DevMu);
    if (m_HostKernel) {
        const std::vector<T> kx = HostKernelRows(x.data(), 1);
        ThrowIfFailed(gprx_model_predict_kx(m_Model, kx.data(), x.data(), 1, mean.data(), D.data()), DefaultContext());
        return mean;
    }
    ThrowIfFailed(gprx_model_predict(m_Model, x.data(), 1, mean.data(), D.data()), DefaultContext());
    return mean;
}

// lib/GaussianProcess.cpp:84-99
template <class T>
T GaussianProcess<T>::operator()(const VectorType& x, const VectorType& y) {
    Initialize();
    CheckInputDimension(x, "GaussianProcess::(): ");
    CheckInputDimension(y, "GaussianProcess::(): ");
    std::lock_guard<std::mutex> lk(m_DevMu);
    EnsureFactor();
    m_CoreSize = m_SampleVectors.size();  // :95-97 builds the core matrix on demand
    T out = 0;
    if (m_HostKernel) {
        const std::vector<T> ka = HostKernelRows(x.data(), 1), kb = HostKernelRows(y.data(), 1);
        const T kab = (*m_Kernel)(x, y);
        ThrowIfFailed(gprx_model_posterior_cov_kx(m_Model, ka.data(), kb.data(), &kab, 1, &out), DefaultContext());
        return out;
    }
    ThrowIfFailed(gprx_model_posterior_cov(m_Model, x.data(), y.data(), 1, &out), DefaultContext());
    return out;
}

// lib/GaussianProcess.cpp:102-114
template <class T>
T GaussianProcess<T>::GetCredibleInterval(const VectorType& x) {
    Initialize();
    CheckInputDimension(x, "GaussianProcess::GetCredibleIntervall: ");
    T c = (*this)(x, x);
    if (debug && c < 0)
        std::cout << "GaussianProcess::GetCredibleIntervall: prediction is instable. gp(x,x) = " << c << "." << std::endl;
    return 2 * std::sqrt(std::max(static_cast<T>(0.0), c));
}

template <class T>
std::vector<T> GaussianProcess<T>::CredibleIntervalBatch(const MatrixType& Xq) {
    Initialize();
    std::lock_guard<std::mutex> lk(m_DevMu);
    EnsureFactor();
    std::vector<T> c(Xq.rows());
    if (m_HostKernel) {
        const std::vector<T> kx = HostKernelRows(Xq.data(), Xq.rows());
        std::vector<T> kk(Xq.rows());
        for (std::size_t a = 0; a < Xq.rows(); a++) kk[a] = (*m_Kernel)(Xq.row(a), Xq.row(a));
        ThrowIfFailed(gprx_model_posterior_cov_kx(m_Model, kx.data(), kx.data(), kk.data(), (int64_t)Xq.rows(), c.data()),
                      DefaultContext());
    } else {
        ThrowIfFailed(gprx_model_posterior_cov(m_Model, Xq.data(), Xq.data(), (int64_t)Xq.rows(), c.data()),
                      DefaultContext());
    }
    for (auto& v : c) v = 2 * std::sqrt(std::max(static_cast<T>(0.0), v));
    return c;
}

// lib/GaussianProcess.cpp:133-180 (same five files, same parameter-file layout including
// the default-precision sigma written before setprecision)
template <class T>
void GaussianProcess<T>::Save(std::string prefix) {
    if (!m_Initialized) throw std::string("GaussianProcess::Save: gaussian process is not initialized.");
    WriteMatrix<MatrixType>(m_RegressionVectors, prefix + "-RegressionVectors.txt");
    if (m_EfficientStorage) {  // :152 drops the in-memory core matrix as well
        m_CoreMatrix.resize(0, 0);
        m_CoreValid = false;
        m_CoreSize = 0;
        WriteMatrix<MatrixType>(MatrixType(0, 0), prefix + "-CoreMatrix.txt");
    } else {
        WriteMatrix<MatrixType>(GetCoreMatrix(), prefix + "-CoreMatrix.txt");
    }
    const std::size_t n = m_SampleVectors.size();
    MatrixType X(m_InputDimension, n), Y(m_OutputDimension, n);
    for (std::size_t i = 0; i < n; i++) {
        for (std::size_t k = 0; k < m_InputDimension; k++) X(k, i) = m_SampleVectors[i][k];
        for (std::size_t c = 0; c < m_OutputDimension; c++) Y(c, i) = m_LabelVectors[i][c];
    }
    WriteMatrix<MatrixType>(X, prefix + "-SampleVectors.txt");
    WriteMatrix<MatrixType>(Y, prefix + "-LabelVectors.txt");
    std::ofstream pf((prefix + "-ParameterFile.txt").c_str());
    pf << m_Sigma << " " << m_InputDimension << " " << m_OutputDimension << " " << m_EfficientStorage << " " << debug
       << " ";
    pf << std::setprecision(std::numeric_limits<T>::digits10 + 1);
    pf << m_Kernel->ToString();
}

// lib/GaussianProcess.cpp:184-268: the loaded regression vectors are used as-is for the
// mean (uploaded next to the samples); the factor is rebuilt on the device on first use.
template <class T>
void GaussianProcess<T>::Load(std::string prefix) {
    const char* names[] = {"-RegressionVectors.txt", "-CoreMatrix.txt", "-SampleVectors.txt", "-LabelVectors.txt",
                           "-ParameterFile.txt"};
    for (const char* nm : names)
        if (!file_ok(prefix + nm))
            throw std::string("GaussianProcess::Load: " + prefix + nm + " does not exist or is a directory.");
    m_RegressionVectors = ReadMatrix<MatrixType>(prefix + "-RegressionVectors.txt");
    m_CoreMatrix = ReadMatrix<MatrixType>(prefix + "-CoreMatrix.txt");
    m_CoreValid = m_CoreMatrix.rows() > 0;
    m_CoreSize = std::min(m_CoreMatrix.rows(), m_CoreMatrix.cols());
    MatrixType X = ReadMatrix<MatrixType>(prefix + "-SampleVectors.txt");
    MatrixType Y = ReadMatrix<MatrixType>(prefix + "-LabelVectors.txt");
    m_SampleVectors.clear();
    m_LabelVectors.clear();
    for (std::size_t i = 0; i < X.cols(); i++) m_SampleVectors.push_back(X.col(i));
    for (std::size_t i = 0; i < Y.cols(); i++) m_LabelVectors.push_back(Y.col(i));
    std::ifstream pf((prefix + "-ParameterFile.txt").c_str());
    std::string line;
    if (std::getline(pf, line)) {
        std::istringstream ls(line);
        if (!(ls >> m_Sigma && ls >> m_InputDimension && ls >> m_OutputDimension && ls >> m_EfficientStorage &&
              ls >> debug))
            throw std::string("GaussianProcess::Load: parameter file is corrupt");
        std::string ks;
        ls >> ks;
        m_Kernel = KernelFactory<T>::GetKernel(ks);
    }
    // the sample lists were replaced: whatever the device held (samples, factor, alpha, a
    // host-evaluated K) belongs to the previous state of this object
    m_DataUploaded = false;
    m_DeviceFactor = false;
    m_HostKernel = false;
    if (m_RegressionVectors.rows() != m_SampleVectors.size() || m_RegressionVectors.cols() != m_OutputDimension)
        throw std::string("GaussianProcess::Load: regression vectors do not match the samples");
    UploadState();
    ThrowIfFailed(gprx_model_set_alpha(m_Model, m_RegressionVectors.data()), DefaultContext());
    m_Initialized = true;
}

template <class T>
void GaussianProcess<T>::ToString() const {
    std::cout << "---------------------------------------" << std::endl;
    std::cout << "Gaussian Process" << std::endl;
    std::cout << " - initialized:\t\t" << m_Initialized << std::endl;
    std::cout << " - # samples:\t\t" << m_SampleVectors.size() << std::endl;
    std::cout << " - # labels:\t\t" << m_LabelVectors.size() << std::endl;
    std::cout << " - noise:\t\t" << m_Sigma << std::endl;
    std::cout << " - input dimension:\t" << m_InputDimension << std::endl;
    std::cout << " - output dimension:\t" << m_OutputDimension << std::endl << std::endl;
    std::cout << " - Kernel:" << std::endl;
    std::cout << "       - Type:\t\t" << m_Kernel->ToString() << std::endl;
    std::cout << "       - Parameter:\t";
    for (const auto& p : m_Kernel->GetStringParameters()) std::cout << p << ", ";
    std::cout << std::endl << "---------------------------------------" << std::endl;
}

// lib/GaussianProcess.cpp:291-360: exact regression-vector match, core matrices compared
// by size only, then samples, labels, kernel, sigma and flags.
template <class T>
bool GaussianProcess<T>::operator==(const GaussianProcess<T>& b) const {
    if (m_RegressionVectors.rows() != b.m_RegressionVectors.rows() ||
        m_RegressionVectors.cols() != b.m_RegressionVectors.cols())
        return false;
    if ((m_RegressionVectors - b.m_RegressionVectors).norm() > 0) return false;
    if (m_CoreSize != b.m_CoreSize) return false;
    if (m_SampleVectors.size() != b.m_SampleVectors.size()) return false;
    for (std::size_t i = 0; i < m_SampleVectors.size(); i++)
        if ((m_SampleVectors[i] - b.m_SampleVectors[i]).norm() > 0) return false;
    if (m_LabelVectors.size() != b.m_LabelVectors.size()) return false;
    for (std::size_t i = 0; i < m_LabelVectors.size(); i++)
        if ((m_LabelVectors[i] - b.m_LabelVectors[i]).norm() > 0) return false;
    if (*m_Kernel != *b.m_Kernel) return false;
    if (m_Sigma != b.m_Sigma) return false;
    if (m_Initialized != b.m_Initialized) return false;
    if (m_InputDimension != b.m_InputDimension || m_OutputDimension != b.m_OutputDimension) return false;
    if (m_EfficientStorage != b.m_EfficientStorage) return false;
    if (debug != b.debug) return false;
    return true;
}

template <class T>
void GaussianProcess<T>::CheckInputDimension(const VectorType& x, std::string msg_prefix) const {
    if (x.size() != m_InputDimension) {
        std::stringstream e;
        e << msg_prefix << "dimension of input vector (" << x.size() << ") does not correspond to the input dimension ("
          << m_InputDimension << ").";
        throw e.str();
    }
}

template <class T>
void GaussianProcess<T>::CheckOutputDimension(const VectorType& y, std::string msg_prefix) const {
    if (y.size() != m_OutputDimension) {
        std::stringstream e;
        e << msg_prefix << "dimension of output vector (" << y.size()
          << ") does not correspond to the output dimension (" << m_OutputDimension << ").";
        throw e.str();
    }
}

template class GaussianProcess<float>;
template class GaussianProcess<double>;

}  // namespace gpr
