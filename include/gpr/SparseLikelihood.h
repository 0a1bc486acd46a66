// gpr/SparseLikelihood.h — SparseLikelihood / SparseGaussianLogLikelihood over libgprx.
//
// Same classes and entry points as the reference (include/SparseLikelihood.h:33-552):
// operator()(gp), GetParameterDerivatives(gp), GetValueAndParameterDerivatives(gp),
// GetValueAndJacobian(gp), taking a GaussianProcess pointer that must be a
// SparseGaussianProcess.  The reference forms the N x N inverse of
// sigma^2 I + Knm Kmm^{-1} Kmn (EfficientInversion, :129-135) and an N x N derivative stack per
// parameter (:246-252); here one device call (gprx_sparse_lml) evaluates the same value and
// gradient in O(N M^2) without them.  The reference's long-double determinant product and its
// clamps (:138-145, 305-314) are reproduced (GPRX_LML_COMPAT), so values match the reference
// where det(C) under/overflows long double.
#pragma once

#include <cmath>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "Likelihood.h"
#include "SparseGaussianProcess.h"

namespace gpr {

template <class TScalarType>
class SparseLikelihood : public Likelihood<TScalarType> {
public:
    typedef Likelihood<TScalarType> Superclass;
    typedef typename Superclass::VectorType VectorType;
    typedef typename Superclass::MatrixType MatrixType;
    typedef typename Superclass::GaussianProcessTypePointer GaussianProcessTypePointer;
    typedef typename Superclass::ValueDerivativePair ValueDerivativePair;
    typedef typename Superclass::ValueJacobianPair ValueJacobianPair;
    typedef SparseGaussianProcess<TScalarType> SparseGaussianProcessType;
    typedef std::shared_ptr<SparseGaussianProcessType> SparseGaussianProcessTypePointer;

    SparseLikelihood() : debug(false) {}
    virtual ~SparseLikelihood() {}
    virtual void DebugOn() { debug = true; }

protected:
    bool debug;
};

// include/SparseLikelihood.h:113-535
template <class TScalarType>
class SparseGaussianLogLikelihood : public SparseLikelihood<TScalarType> {
public:
    typedef SparseLikelihood<TScalarType> Superclass;
    typedef SparseGaussianLogLikelihood Self;
    typedef std::shared_ptr<Self> Pointer;
    typedef typename Superclass::VectorType VectorType;
    typedef typename Superclass::MatrixType MatrixType;
    typedef typename Superclass::GaussianProcessTypePointer GaussianProcessTypePointer;
    typedef typename Superclass::SparseGaussianProcessTypePointer SparseGaussianProcessTypePointer;
    typedef typename Superclass::ValueDerivativePair ValueDerivativePair;
    typedef typename Superclass::ValueJacobianPair ValueJacobianPair;

    SparseGaussianLogLikelihood() {}
    virtual ~SparseGaussianLogLikelihood() {}

    // :148-216
    virtual VectorType operator()(const GaussianProcessTypePointer gp) const {
        double v = 0, ld = 0;
        CastToSparseGaussianProcess(gp)->EvaluateLogLikelihood(false, true, &v, nullptr, &ld);
        return Value(v);
    }
    // :218-283
    virtual VectorType GetParameterDerivatives(const GaussianProcessTypePointer gp) const {
        double v = 0, ld = 0;
        std::vector<double> g;
        CastToSparseGaussianProcess(gp)->EvaluateLogLikelihood(true, true, &v, &g, &ld);
        return Grad(g);
    }
    // :285-414
    virtual ValueDerivativePair GetValueAndParameterDerivatives(const GaussianProcessTypePointer gp) const {
        double v = 0, ld = 0;
        std::vector<double> g;
        CastToSparseGaussianProcess(gp)->EvaluateLogLikelihood(true, true, &v, &g, &ld);
        return std::make_pair(Value(v), Grad(g));
    }
    // :416-535: one label column, so the Jacobian is the gradient as a 1 x P row
    virtual ValueJacobianPair GetValueAndJacobian(const GaussianProcessTypePointer gp) const {
        double v = 0, ld = 0;
        std::vector<double> g;
        CastToSparseGaussianProcess(gp)->EvaluateLogLikelihood(true, true, &v, &g, &ld);
        MatrixType J(1, g.size());
        for (std::size_t p = 0; p < g.size(); p++) J(0, p) = (TScalarType)g[p];
        return std::make_pair(Value(v), J);
    }
    virtual std::string ToString() const { return "SparseGaussianLogLikelihood"; }

private:
    static SparseGaussianProcessTypePointer CastToSparseGaussianProcess(const GaussianProcessTypePointer gp) {
        SparseGaussianProcessTypePointer sgp(
            std::dynamic_pointer_cast<SparseGaussianProcess<TScalarType>>(gp));
        if (sgp.get() == nullptr) throw std::string("SparseGaussianLogLikelihood: cannot cast to SparseGaussianProcess");
        return sgp;
    }
    static VectorType Value(double v) {
        VectorType out(1);
        out[0] = (TScalarType)v;
        return out;
    }
    static VectorType Grad(const std::vector<double>& g) {
        VectorType out(g.size());
        for (std::size_t p = 0; p < g.size(); p++) out[p] = (TScalarType)g[p];
        return out;
    }
    SparseGaussianLogLikelihood(const Self&) = delete;
    void operator=(const Self&) = delete;
};

}  // namespace gpr
