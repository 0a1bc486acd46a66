// gpr/GaussianProcessInference.h — GaussianProcessInference<T>: the reference's maximum-
// likelihood loop over the kernel parameters (include/GaussianProcessInference.h:38-243), on
// the device-resident GP.
//
// Same constructor, GetParameters, SetParametersToOptimize, Optimize (Gauss-Newton on the
// rank-1 system g g^T with log-damped steps, :84-159) and Optimize2 (Gauss-Newton on J^T J,
// :161-229).  Each iteration sets the kernel parameters and calls the likelihood's
// GetValueAndParameterDerivatives / GetValueAndJacobian: one device call that refits the
// factor and evaluates value and gradient (gprx_model_lml, or gprx_sparse_lml for a
// SparseGaussianProcess with SparseGaussianLogLikelihood).  The samples stay in HBM across
// iterations (GaussianProcess::UploadState re-sends only the kernel).  pinv is the reference's
// SVD pseudo-inverse (include/Prior.h:38-55: singular values <= epsilon dropped), computed by
// one-sided Jacobi on the P x P host matrix.
#pragma once

#include <algorithm>
#include <cmath>
#include <iostream>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "GaussianProcess.h"
#include "Likelihood.h"

namespace gpr {

// Moore-Penrose pseudo-inverse of a square matrix through its SVD (include/Prior.h:38-55):
// one-sided Jacobi rotations orthogonalise the columns of A V, the column norms are the
// singular values, pinv = V diag(1/s_i for s_i > epsilon, else 0) U^T.
template <class TMatrixType>
TMatrixType pinv(const TMatrixType& m, double epsilon = std::numeric_limits<double>::epsilon()) {
    const std::size_t r = m.rows(), c = m.cols();
    std::vector<double> A(r * c), V(c * c, 0.0);
    for (std::size_t i = 0; i < r; i++)
        for (std::size_t j = 0; j < c; j++) A[i * c + j] = (double)m(i, j);
    for (std::size_t j = 0; j < c; j++) V[j * c + j] = 1.0;
    for (int sweep = 0; sweep < 60; sweep++) {
        double off = 0;
        for (std::size_t p = 0; p + 1 < c; p++)
            for (std::size_t q = p + 1; q < c; q++) {
                double app = 0, aqq = 0, apq = 0;
                for (std::size_t i = 0; i < r; i++) {
                    app += A[i * c + p] * A[i * c + p];
                    aqq += A[i * c + q] * A[i * c + q];
                    apq += A[i * c + p] * A[i * c + q];
                }
                if (apq == 0.0 || std::fabs(apq) <= 1e-300) continue;
                off = std::max(off, std::fabs(apq) / std::sqrt(std::max(app * aqq, 1e-300)));
                const double zeta = (aqq - app) / (2 * apq);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1 + zeta * zeta));
                const double cs = 1 / std::sqrt(1 + t * t), sn = cs * t;
                for (std::size_t i = 0; i < r; i++) {
                    const double x = A[i * c + p], y = A[i * c + q];
                    A[i * c + p] = cs * x - sn * y;
                    A[i * c + q] = sn * x + cs * y;
                }
                for (std::size_t i = 0; i < c; i++) {
                    const double x = V[i * c + p], y = V[i * c + q];
                    V[i * c + p] = cs * x - sn * y;
                    V[i * c + q] = sn * x + cs * y;
                }
            }
        if (off < 1e-15) break;
    }
    // column j of A V = s_j u_j
    TMatrixType out(c, r);
    std::vector<double> s(c), inv(c);
    for (std::size_t j = 0; j < c; j++) {
        double nrm = 0;
        for (std::size_t i = 0; i < r; i++) nrm += A[i * c + j] * A[i * c + j];
        s[j] = std::sqrt(nrm);
        inv[j] = (s[j] <= epsilon) ? 0.0 : 1.0 / s[j];
    }
    for (std::size_t a = 0; a < c; a++)
        for (std::size_t b = 0; b < r; b++) {
            double acc = 0;  // sum_j V[a][j] inv_j u_j[b],  u_j[b] = A[b][j] / s_j
            for (std::size_t j = 0; j < c; j++)
                if (inv[j] != 0.0) acc += V[a * c + j] * inv[j] * (A[b * c + j] * inv[j]);
            out(a, b) = (typename std::remove_reference<decltype(out(a, b))>::type)acc;
        }
    return out;
}

template <class TScalarType>
class GaussianProcessInference {
public:
    typedef GaussianProcessInference Self;
    typedef std::shared_ptr<Self> Pointer;
    typedef GaussianProcess<TScalarType> GaussianProcessType;
    typedef typename GaussianProcessType::Pointer GaussianProcessTypePointer;
    typedef typename GaussianProcessType::VectorType VectorType;
    typedef typename GaussianProcessType::MatrixType MatrixType;
    typedef std::vector<TScalarType> ParameterVectorType;
    typedef std::vector<bool> BooleanVectorType;
    typedef Likelihood<TScalarType> LikelihoodType;
    typedef typename LikelihoodType::Pointer LikelihoodTypePointer;
    typedef typename LikelihoodType::ValueDerivativePair ValueDerivativePair;
    typedef typename LikelihoodType::ValueJacobianPair ValueJacobianPair;

    // :59-69
    GaussianProcessInference(LikelihoodTypePointer lh, GaussianProcessTypePointer gp, double stepwidth,
                             unsigned iterations)
        : m_StepWidth(stepwidth),
          m_StepWidth3(stepwidth * stepwidth * stepwidth),
          m_NumberOfIterations(iterations),
          m_Likelihood(lh),
          m_GaussianProcess(gp) {
        m_Parameters = m_GaussianProcess->GetKernel()->GetParameters();
        for (std::size_t i = 0; i < m_Parameters.size(); i++) m_ParametersToOptimize.push_back(true);
    }
    ~GaussianProcessInference() {}

    ParameterVectorType GetParameters() { return m_Parameters; }

    // :77-81
    void SetParametersToOptimize(const BooleanVectorType& v) {
        for (std::size_t i = 0; i < std::min(m_ParametersToOptimize.size(), v.size()); i++)
            m_ParametersToOptimize[i] = v[i];
    }

    // :84-159
    void Optimize(bool output = true, bool exp_output = false) {
        for (unsigned i = 0; i < m_NumberOfIterations; i++) {
            try {
                m_GaussianProcess->GetKernel()->SetParameters(m_Parameters);
                ValueDerivativePair vd = m_Likelihood->GetValueAndParameterDerivatives(m_GaussianProcess);
                const VectorType& g = vd.second;
                const VectorType& likelihood = vd.first;
                const double sign = (likelihood[0] > 0) ? -1 : 1;
                const std::size_t P = g.size();
                MatrixType ggt(P, P);
                for (std::size_t a = 0; a < P; a++)
                    for (std::size_t b = 0; b < P; b++) ggt(a, b) = g[a] * g[b];
                const MatrixType pi = pinv<MatrixType>(ggt);
                VectorType update(P);
                for (std::size_t a = 0; a < P; a++) {
                    TScalarType acc = 0;
                    for (std::size_t b = 0; b < P; b++) acc += pi(a, b) * g[b];
                    update[a] = acc;
                }
                if (output) Report(likelihood[0], exp_output, ", Gradients: ", g, ", inf(J'J)J': ", update);
                for (std::size_t p = 0; p < m_Parameters.size(); p++) {
                    double u;
                    if (update[p] == 0) {  // log gradient step
                        u = (g[p] >= 0) ? m_StepWidth3 * std::log(1 + g[p]) : -m_StepWidth3 * std::log(1 + std::fabs(g[p]));
                        m_Parameters[p] += u * sign;
                    } else {  // Gauss Newton step
                        u = update[p] * likelihood[0];
                        u = (u > 0) ? m_StepWidth * std::log(1 + u) : -m_StepWidth * std::log(1 + std::fabs(u));
                        m_Parameters[p] -= u * sign;
                    }
                    if (output) std::cout << u << " " << std::flush;
                }
                if (output) ReportParameters(exp_output);
            } catch (std::string& s) {
                std::cout << "[failed] " << s << std::endl;
                return;
            }
        }
    }

    // :161-229
    void Optimize2(bool output = true, bool exp_output = false) {
        VectorType old_likelihood;
        for (unsigned i = 0; i < m_NumberOfIterations; i++) {
            try {
                m_GaussianProcess->GetKernel()->SetParameters(m_Parameters);
                ValueJacobianPair vj = m_Likelihood->GetValueAndJacobian(m_GaussianProcess);
                const MatrixType& J = vj.second;
                VectorType likelihood = vj.first;
                if (i == 0) {
                    old_likelihood = likelihood;
                } else {
                    double d2 = 0;
                    for (std::size_t l = 0; l < likelihood.size(); l++)
                        d2 += (double)(old_likelihood[l] - likelihood[l]) * (double)(old_likelihood[l] - likelihood[l]);
                    if (d2 == 0) break;
                }
                for (std::size_t l = 0; l < likelihood.size(); l++) {
                    const double sign = (likelihood[l] > 0) ? -1 : 1;
                    likelihood[l] *= sign;
                }
                const std::size_t L = J.rows(), P = J.cols();
                MatrixType JtJ(P, P);
                for (std::size_t a = 0; a < P; a++)
                    for (std::size_t b = 0; b < P; b++) {
                        TScalarType acc = 0;
                        for (std::size_t l = 0; l < L; l++) acc += J(l, a) * J(l, b);
                        JtJ(a, b) = acc;
                    }
                const MatrixType pi = pinv<MatrixType>(JtJ);
                VectorType Jtl(P), update(P);
                for (std::size_t a = 0; a < P; a++) {
                    TScalarType acc = 0;
                    for (std::size_t l = 0; l < L; l++) acc += J(l, a) * likelihood[l];
                    Jtl[a] = acc;
                }
                for (std::size_t a = 0; a < P; a++) {
                    TScalarType acc = 0;
                    for (std::size_t b = 0; b < P; b++) acc += pi(a, b) * Jtl[b];
                    update[a] = acc;
                }
                if (output) {
                    VectorType dj(std::min(L, P));
                    for (std::size_t a = 0; a < dj.size(); a++) dj[a] = J(a, a);
                    Report(vj.first[0], exp_output, ", diag(J): ", dj, ", update: ", update);
                }
                for (std::size_t p = 0; p < m_Parameters.size(); p++) {
                    if (!m_ParametersToOptimize[p]) continue;
                    if (update[p] > 0) m_Parameters[p] -= m_StepWidth * std::log(1 + update[p]);
                    else m_Parameters[p] -= -m_StepWidth * std::log(1 + std::fabs(update[p]));
                }
                if (output) ReportParameters(exp_output);
                old_likelihood = likelihood;
            } catch (std::string& s) {
                std::cout << "[failed] " << s << std::endl;
                return;
            }
        }
    }

private:
    void Report(double lik, bool exp_output, const char* l1, const VectorType& a, const char* l2,
                const VectorType& b) const {
        std::cout << "Likelihood " << lik << ", : ";
        for (std::size_t p = 0; p < m_Parameters.size(); p++)
            std::cout << (exp_output ? std::exp(m_Parameters[p]) : m_Parameters[p]) << ", ";
        std::cout << l1;
        for (std::size_t p = 0; p < a.size(); p++) std::cout << a[p] << " ";
        std::cout << l2;
        for (std::size_t p = 0; p < b.size(); p++) std::cout << b[p] << " ";
        std::cout << ", update: " << std::flush;
    }
    void ReportParameters(bool exp_output) const {
        std::cout << ", new parameters: ";
        for (std::size_t p = 0; p < m_Parameters.size(); p++)
            std::cout << (exp_output ? std::exp(m_Parameters[p]) : m_Parameters[p]) << ", ";
        std::cout << std::endl;
    }

    TScalarType m_StepWidth;
    TScalarType m_StepWidth3;
    unsigned m_NumberOfIterations;
    BooleanVectorType m_ParametersToOptimize;
    LikelihoodTypePointer m_Likelihood;
    GaussianProcessTypePointer m_GaussianProcess;
    ParameterVectorType m_Parameters;

    GaussianProcessInference(const Self&) = delete;
    void operator=(const Self&) = delete;
};

}  // namespace gpr
