// gpr/Likelihood.h — GaussianLikelihood / GaussianLogLikelihood over libgprx.
//
// Same classes and entry points as the reference (include/Likelihood.h:34-354):
// operator()(gp), GetParameterDerivatives(gp), GetValueAndParameterDerivatives(gp),
// GetValueAndJacobian(gp).  The reference forms C = (K + sigma^2 I)^{-1} explicitly and the
// determinant through a long-double LU; here one device call (gprx_model_lml) refits the
// factor and evaluates value and gradient from it.  GPRX_LML_COMPAT reproduces the
// reference's narrowing of the determinant to T and its clamps (Likelihood.h:77-79,
// 240-257) so values match the reference where det(K) under/overflows T.
#pragma once

#include <cmath>
#include <limits>
#include <sstream>
#include <string>
#include <utility>

#include "GaussianProcess.h"

namespace gpr {

template <class TScalarType>
class Likelihood {
public:
    typedef Likelihood Self;
    typedef std::shared_ptr<Self> Pointer;
    typedef GaussianProcess<TScalarType> GaussianProcessType;
    typedef std::shared_ptr<GaussianProcessType> GaussianProcessTypePointer;
    typedef typename GaussianProcessType::VectorType VectorType;
    typedef typename GaussianProcessType::MatrixType MatrixType;
    typedef std::pair<VectorType, VectorType> ValueDerivativePair;
    typedef std::pair<VectorType, MatrixType> ValueJacobianPair;
    typedef long double HighPrecisionType;

    virtual VectorType operator()(const GaussianProcessTypePointer) const {
        throw std::string("Likelihood: operator() is not implemented.");
    }
    virtual VectorType GetParameterDerivatives(const GaussianProcessTypePointer) const {
        throw std::string("Likelihood: GetParameterDerivatives is not implemented.");
    }
    virtual ValueDerivativePair GetValueAndParameterDerivatives(const GaussianProcessTypePointer) const {
        throw std::string("Likelihood: GetValueAndParameterDerivatives is not implemented.");
    }
    virtual ValueJacobianPair GetValueAndJacobian(const GaussianProcessTypePointer) const {
        throw std::string("Likelihood: GetValueAndJacobian is not implemented.");
    }
    virtual std::string ToString() const = 0;
    virtual ~Likelihood() {}

protected:
    // One device evaluation on the gp's current samples/kernel/noise (the reference
    // re-runs ComputeCoreMatrix in GetCoreMatrix, include/Likelihood.h:77-79).
    struct Eval {
        double value = 0, logdet = 0;
        std::vector<double> grad;
    };
    Eval Evaluate(const GaussianProcessTypePointer gp, bool grad, bool compat = true) const {
        // the kernel swap, the likelihood's refit and the alpha restore are one step for a
        // concurrent Predict / operator() on the same gp (they take m_DevMu too)
        std::lock_guard<std::mutex> lk(gp->m_DevMu);
        gp->UploadState();
        if (gp->m_OutputDimension != 1)
            throw std::string("GaussianLogLikelihood: device likelihood supports one output dimension");
        Eval e;
        int32_t np = 0;
        e.grad.resize(GPRX_MAX_KNODES * 3);
        uint32_t flags = (compat ? GPRX_LML_COMPAT : 0u) | (grad ? GPRX_LML_GRAD : 0u);
        typedef GaussianProcess<TScalarType> GPT;
        if (gp->m_InvMethod == GPT::JacobiSVD || gp->m_InvMethod == GPT::BDCSVD) flags |= GPRX_LML_FORCE_LU;
        if (gp->m_HostKernel) {  // no device form: the derivative matrices through GetDerivative
            std::vector<TScalarType> dK;
            if (grad) dK = gp->HostDerivativeMatrices(np);
            if ((int32_t)e.grad.size() < np) e.grad.resize(np);
            ThrowIfFailed(gprx_model_lml_dk(gp->m_Model, flags & ~GPRX_LML_GRAD, grad ? dK.data() : nullptr,
                                            grad ? np : 0, &e.value, grad ? e.grad.data() : nullptr, &e.logdet),
                          DefaultContext());
        } else {
            ThrowIfFailed(gprx_model_lml(gp->m_Model, flags, &e.value, grad ? e.grad.data() : nullptr, &np, &e.logdet),
                          DefaultContext());
        }
        gp->m_DeviceFactor = true;
        gp->m_CoreValid = false;
        // the likelihood does not change the gp's regression vectors (the reference only
        // reads its core matrix): keep predicting with them
        if (gp->m_Initialized && gp->m_RegressionVectors.rows() == gp->m_SampleVectors.size())
            ThrowIfFailed(gprx_model_set_alpha(gp->m_Model, gp->m_RegressionVectors.data()), DefaultContext());
        e.grad.resize(np);
        return e;
    }
};

// include/Likelihood.h:94-150: exp(data fit) / sqrt(det) / (2 pi)^{N/2}
template <class TScalarType>
class GaussianLikelihood : public Likelihood<TScalarType> {
public:
    typedef Likelihood<TScalarType> Superclass;
    typedef typename Superclass::VectorType VectorType;
    typedef typename Superclass::GaussianProcessTypePointer GaussianProcessTypePointer;
    typedef typename Superclass::HighPrecisionType HighPrecisionType;

    GaussianLikelihood() {}
    virtual VectorType operator()(const GaussianProcessTypePointer gp) const {
        auto e = this->Evaluate(gp, false, false);
        const double n = gp->GetNumberOfSamples();
        // exact value = df - logdet/2 - n/2 log(2pi); recover the data fit df
        const double df = e.value + 0.5 * e.logdet + n / 2.0 * std::log(2 * M_PI);
        // the reference's determinant is narrowed to T (include/Likelihood.h:77-79)
        const HighPrecisionType det = (HighPrecisionType)(TScalarType)std::exp((long double)e.logdet);
        if (det < -std::numeric_limits<HighPrecisionType>::epsilon()) {
            std::stringstream ss;
            ss << "GaussianLikelihood: determinant of K is smaller than zero: " << det;
            throw ss.str();
        }
        TScalarType cp = det <= 0 ? TScalarType(1.0 / std::sqrt(std::numeric_limits<HighPrecisionType>::min()))
                                  : TScalarType(1.0 / std::sqrt(det));
        TScalarType ct = TScalarType(1.0 / std::pow(2 * M_PI, n / 2.0));
        VectorType v(1);
        v[0] = TScalarType(std::exp(df)) * cp * ct;
        return v;
    }
    virtual std::string ToString() const { return "GaussianLikelihood"; }
};

// include/Likelihood.h:152-354
template <class TScalarType>
class GaussianLogLikelihood : public Likelihood<TScalarType> {
public:
    typedef Likelihood<TScalarType> Superclass;
    typedef typename Superclass::VectorType VectorType;
    typedef typename Superclass::MatrixType MatrixType;
    typedef typename Superclass::GaussianProcessTypePointer GaussianProcessTypePointer;
    typedef typename Superclass::ValueDerivativePair ValueDerivativePair;
    typedef typename Superclass::ValueJacobianPair ValueJacobianPair;

    GaussianLogLikelihood() {}
    virtual VectorType operator()(const GaussianProcessTypePointer gp) const {
        auto e = this->Evaluate(gp, false);
        return Value(e);
    }
    virtual VectorType GetParameterDerivatives(const GaussianProcessTypePointer gp) const {
        return Grad(this->Evaluate(gp, true));
    }
    virtual ValueDerivativePair GetValueAndParameterDerivatives(const GaussianProcessTypePointer gp) const {
        auto e = this->Evaluate(gp, true);
        return std::make_pair(Value(e), Grad(e));
    }
    // one output column (m = 1): the Jacobian is the gradient as a 1 x P row
    virtual ValueJacobianPair GetValueAndJacobian(const GaussianProcessTypePointer gp) const {
        auto e = this->Evaluate(gp, true);
        VectorType g = Grad(e);
        MatrixType J(1, g.size());
        for (std::size_t p = 0; p < g.size(); p++) J(0, p) = g[p];
        return std::make_pair(Value(e), J);
    }
    virtual std::string ToString() const { return "GaussianLogLikelihood"; }

private:
    static VectorType Value(const typename Superclass::Eval& e) {
        if (std::isinf(e.value))
            throw std::string("GaussianLogLikelihood::GetValueAndParameterDerivatives: likelihood is infinite.");
        VectorType v(1);
        v[0] = (TScalarType)e.value;
        return v;
    }
    static VectorType Grad(const typename Superclass::Eval& e) {
        VectorType g(e.grad.size());
        for (std::size_t p = 0; p < e.grad.size(); p++) g[p] = (TScalarType)e.grad[p];
        return g;
    }
};

}  // namespace gpr
