// gpr/Kernel.h — the Kernel<T> hierarchy of the host API.
//
// Same classes, constructors, parameter order, string form and validation behaviour as the
// reference (include/Kernel.h:40-1036): Kernel<T> with virtual operator()(x,y) and
// GetDerivative(x,y); leaves GaussianKernel (sigma, scale), GaussianExpKernel (sigma,
// scale), WhiteKernel (scale), RationalQuadraticKernel (scale, sigma, alpha),
// PeriodicKernel (scale, b, sigma); composites SumKernel / ProductKernel.
//
// operator() / GetDerivative evaluate ONE pair on the host (the reference's scalar API).
// Matrix-shaped work never calls them: every kernel lowers itself with Describe() into the
// post-order gprx_kernel_desc program that libgprx evaluates on the GPU.  A user subclass
// that does not override Describe() cannot be used by GaussianProcess (it throws).
#pragma once

#include <cmath>
#include <iomanip>
#include <limits>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "../gprx.h"
#include "Matrix.h"

namespace gpr {

template <class T>
class Kernel {
public:
    typedef Kernel Self;
    typedef std::shared_ptr<Self> Pointer;
    typedef DenseVector<T> VectorType;
    typedef std::vector<T> ParameterVectorType;
    typedef std::string StringParameterType;
    typedef std::vector<StringParameterType> StringParameterVectorType;

    Kernel() {}
    virtual ~Kernel() {}
    Kernel(const Self&) = delete;
    void operator=(const Self&) = delete;

    virtual T operator()(const VectorType& x, const VectorType& y) const {
        (void)x;
        (void)y;
        throw std::string("Kernel: operator() is not implemented.");
    }
    virtual VectorType GetDerivative(const VectorType& x, const VectorType& y) const {
        (void)x;
        (void)y;
        throw std::string("Kernel: GetDerivative() is not implemented.");
    }
    virtual std::string ToString() const = 0;
    virtual unsigned GetNumberOfParameters() const = 0;
    virtual const StringParameterVectorType GetStringParameters() const { return m_StringParameters; }
    virtual ParameterVectorType GetParameters() const { return m_Parameters; }
    virtual void SetParameters(const ParameterVectorType& parameters) = 0;

    // Lowering to the device program (post-order).  Not in the reference: this is the
    // contract between the host classes and libgprx.
    virtual void Describe(std::vector<gprx_knode>& prog) const {
        (void)prog;
        throw std::string("Kernel: " + ToString() + " has no device form (override Kernel::Describe).");
    }

    std::string ParametersToString(const StringParameterVectorType& params) const {
        std::string s;
        for (const auto& p : params) s += p + ",";
        return s;
    }

    // include/Kernel.h:93-114: same string, string parameters and parameters within 10 eps
    virtual bool operator==(const Kernel<T>& b) const {
        if (ToString() != b.ToString()) return false;
        if (m_StringParameters != b.m_StringParameters) return false;
        if (m_Parameters.size() != b.m_Parameters.size()) return false;
        for (std::size_t i = 0; i < m_Parameters.size(); i++)
            if (std::fabs(m_Parameters[i] - b.m_Parameters[i]) > 10 * std::numeric_limits<T>::epsilon()) return false;
        return true;
    }
    virtual bool operator!=(const Kernel<T>& b) const { return !operator==(b); }

protected:
    ParameterVectorType m_Parameters;
    StringParameterVectorType m_StringParameters;

    static std::string P2S(T p) {  // maximal-precision scalar -> string (include/Kernel.h:127-132)
        std::ostringstream ss;
        ss << std::setprecision(std::numeric_limits<T>::digits10 + 1) << p;
        return ss.str();
    }
    static T S2P(const std::string& s) {
        T p;
        std::istringstream ss(s);
        ss >> p;
        return p;
    }
    static T dist2(const VectorType& x, const VectorType& y) {
        if (x.size() != y.size()) throw std::string("Kernel: input vectors of different dimension.");
        T r = (x - y).norm();
        return r * r;  // the reference squares the norm (include/Kernel.h:466-467)
    }
    static void push_leaf(std::vector<gprx_knode>& prog, int op, const ParameterVectorType& p) {
        gprx_knode n{};
        n.op = op;
        for (std::size_t i = 0; i < p.size() && i < 3; i++) n.p[i] = (double)p[i];
        prog.push_back(n);
    }
};

// ------------------------------------------------------------------------------------
// Leaves.  Each stores its parameters in reference order and recomputes the derived
// constants in SetParameters.  Validation reproduces the reference quirk of checking the
// values held BEFORE the assignment (include/Kernel.h:529-533, 1003-1008).
// ------------------------------------------------------------------------------------
template <class T>
class GaussianKernel : public Kernel<T> {
public:
    typedef Kernel<T> Superclass;
    typedef std::shared_ptr<GaussianKernel> Pointer;
    using typename Superclass::VectorType;
    using typename Superclass::ParameterVectorType;
    using typename Superclass::StringParameterVectorType;

    GaussianKernel(T sigma, T scale = 1) : m_Sigma(sigma), m_Scale(scale) { Assign({sigma, scale}); }
    GaussianKernel(const std::string& p1, const std::string& p2) : GaussianKernel(this->S2P(p1), this->S2P(p2)) {}

    T operator()(const VectorType& x, const VectorType& y) const override {
        return m_Scale * m_Scale * std::exp(-0.5 * this->dist2(x, y) / (m_Sigma * m_Sigma));
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        const T r2 = this->dist2(x, y);
        const T f = std::exp(-0.5 * r2 / (m_Sigma * m_Sigma));
        VectorType D(2);
        D[0] = m_Scale * m_Scale * r2 / (m_Sigma * m_Sigma * m_Sigma) * f;
        D[1] = 2 * m_Scale * f;
        return D;
    }
    std::string ToString() const override { return "GaussianKernel(" + this->ParametersToString(this->m_StringParameters) + ")"; }
    unsigned GetNumberOfParameters() const override { return 2; }
    void SetParameters(const ParameterVectorType& p) override {
        if (p.size() != 2) throw std::string("GaussianKernel::SetParameters: wrong number of parameters.");
        Assign(p);
    }
    static Pointer Load(const StringParameterVectorType& p) {
        if (p.size() != 2) throw std::string("GaussianKernel::Load: wrong number of kernel parameters.");
        return Pointer(new GaussianKernel(Superclass::S2P(p[0]), Superclass::S2P(p[1])));
    }
    void Describe(std::vector<gprx_knode>& prog) const override { this->push_leaf(prog, GPRX_K_GAUSSIAN, this->m_Parameters); }

private:
    void Assign(const ParameterVectorType& p) {
        if (m_Sigma == 0) throw std::string("GaussianKernel: sigma has to be positive");
        if (m_Scale == 0) throw std::string("GaussianKernel: scale has to be positive");
        m_Sigma = p[0];
        m_Scale = p[1];
        this->m_Parameters = p;
        this->m_StringParameters = {this->P2S(m_Sigma), this->P2S(m_Scale)};
    }
    T m_Sigma, m_Scale;
};

template <class T>
class GaussianExpKernel : public Kernel<T> {
public:
    typedef Kernel<T> Superclass;
    typedef std::shared_ptr<GaussianExpKernel> Pointer;
    using typename Superclass::VectorType;
    using typename Superclass::ParameterVectorType;
    using typename Superclass::StringParameterVectorType;

    GaussianExpKernel(T sigma, T scale = 1) { Assign({sigma, scale}); }
    GaussianExpKernel(const std::string& p1, const std::string& p2) : GaussianExpKernel(this->S2P(p1), this->S2P(p2)) {}

    T operator()(const VectorType& x, const VectorType& y) const override {
        const T es = std::exp(m_Scale), eg = std::exp(m_Sigma);
        return es * es * std::exp(-0.5 * this->dist2(x, y) / (eg * eg));
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        const T r2 = this->dist2(x, y);
        const T f1 = std::exp(-2 * m_Sigma), f2 = std::exp(2 * m_Sigma);
        VectorType D(2);
        D[0] = r2 * std::exp(-0.5 * f1 * ((4 * m_Sigma - 4 * m_Scale) * f2 + r2));
        D[1] = 2 * std::exp(0.5 * f1 * (4 * f2 * m_Scale - r2));
        return D;
    }
    std::string ToString() const override { return "GaussianExpKernel(" + this->ParametersToString(this->m_StringParameters) + ")"; }
    unsigned GetNumberOfParameters() const override { return 2; }
    void SetParameters(const ParameterVectorType& p) override {
        if (p.size() != 2) throw std::string("GaussianExpKernel::SetParameters: wrong number of parameters.");
        Assign(p);
    }
    static Pointer Load(const StringParameterVectorType& p) {
        if (p.size() != 2) throw std::string("GaussianExpKernel::Load: wrong number of kernel parameters.");
        return Pointer(new GaussianExpKernel(Superclass::S2P(p[0]), Superclass::S2P(p[1])));
    }
    void Describe(std::vector<gprx_knode>& prog) const override { this->push_leaf(prog, GPRX_K_GAUSSIAN_EXP, this->m_Parameters); }

private:
    void Assign(const ParameterVectorType& p) {
        m_Sigma = p[0];
        m_Scale = p[1];
        this->m_Parameters = p;
        this->m_StringParameters = {this->P2S(m_Sigma), this->P2S(m_Scale)};
    }
    T m_Sigma = 0, m_Scale = 0;
};

template <class T>
class WhiteKernel : public Kernel<T> {
public:
    typedef Kernel<T> Superclass;
    typedef std::shared_ptr<WhiteKernel> Pointer;
    using typename Superclass::VectorType;
    using typename Superclass::ParameterVectorType;
    using typename Superclass::StringParameterVectorType;

    explicit WhiteKernel(T scale) { Assign({scale}); }
    explicit WhiteKernel(const std::string& p1) : WhiteKernel(this->S2P(p1)) {}

    T operator()(const VectorType& x, const VectorType& y) const override {
        return ((x - y).norm() == 0) ? m_Scale * m_Scale : T(0);
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        VectorType D(1);
        D[0] = ((x - y).norm() == 0) ? 2 * m_Scale : T(0);
        return D;
    }
    std::string ToString() const override { return "WhiteKernel(" + this->ParametersToString(this->m_StringParameters) + ")"; }
    unsigned GetNumberOfParameters() const override { return 1; }
    void SetParameters(const ParameterVectorType& p) override {
        if (p.size() != 1) throw std::string("WhiteKernel::SetParameters: wrong number of parameters.");
        Assign(p);
    }
    static Pointer Load(const StringParameterVectorType& p) {
        if (p.size() != 1) throw std::string("WhiteKernel::Load: wrong number of kernel parameters.");
        return Pointer(new WhiteKernel(Superclass::S2P(p[0])));
    }
    void Describe(std::vector<gprx_knode>& prog) const override { this->push_leaf(prog, GPRX_K_WHITE, this->m_Parameters); }

private:
    void Assign(const ParameterVectorType& p) {
        m_Scale = p[0];
        this->m_Parameters = p;
        this->m_StringParameters = {this->P2S(m_Scale)};
    }
    T m_Scale = 0;
};

template <class T>
class RationalQuadraticKernel : public Kernel<T> {
public:
    typedef Kernel<T> Superclass;
    typedef std::shared_ptr<RationalQuadraticKernel> Pointer;
    using typename Superclass::VectorType;
    using typename Superclass::ParameterVectorType;
    using typename Superclass::StringParameterVectorType;

    RationalQuadraticKernel(T scale, T sigma, T alpha) { Assign({scale, sigma, alpha}); }
    RationalQuadraticKernel(const std::string& p1, const std::string& p2, const std::string& p3)
        : RationalQuadraticKernel(this->S2P(p1), this->S2P(p2), this->S2P(p3)) {}

    T operator()(const VectorType& x, const VectorType& y) const override {
        return m_Scale * m_Scale * std::pow(1 + 0.5 * this->dist2(x, y) / (m_Sigma * m_Sigma * m_Alpha), -m_Alpha);
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        const T r2 = this->dist2(x, y);
        const T s2 = m_Sigma * m_Sigma;
        const T f = 0.5 * r2 / (s2 * m_Alpha) + 1;
        VectorType D(3);
        D[0] = 2 * m_Scale * std::pow(f, -m_Alpha);
        D[1] = m_Scale * m_Scale * r2 * std::pow(f, -m_Alpha - 1) / (s2 * m_Sigma);
        D[2] = m_Scale * m_Scale * ((r2 / (2 * s2 * f * m_Alpha)) - std::log(f)) * std::pow(f, -m_Alpha);
        return D;
    }
    std::string ToString() const override {
        return "RationalQuadraticKernel(" + this->ParametersToString(this->m_StringParameters) + ")";
    }
    unsigned GetNumberOfParameters() const override { return 3; }
    void SetParameters(const ParameterVectorType& p) override {
        if (p.size() != 3) throw std::string("RationalQuadraticKernel::SetParameters: wrong number of parameters.");
        Assign(p);
    }
    static Pointer Load(const StringParameterVectorType& p) {
        if (p.size() != 3) throw std::string("RationalQuadraticKernel::Load: wrong number of kernel parameters.");
        return Pointer(new RationalQuadraticKernel(Superclass::S2P(p[0]), Superclass::S2P(p[1]), Superclass::S2P(p[2])));
    }
    void Describe(std::vector<gprx_knode>& prog) const override {
        this->push_leaf(prog, GPRX_K_RATIONAL_QUADRATIC, this->m_Parameters);
    }

private:
    void Assign(const ParameterVectorType& p) {
        m_Scale = p[0];
        m_Sigma = p[1];
        m_Alpha = p[2];
        this->m_Parameters = p;
        this->m_StringParameters = {this->P2S(m_Scale), this->P2S(m_Sigma), this->P2S(m_Alpha)};
    }
    T m_Scale = 0, m_Sigma = 0, m_Alpha = 0;
};

template <class T>
class PeriodicKernel : public Kernel<T> {
public:
    typedef Kernel<T> Superclass;
    typedef std::shared_ptr<PeriodicKernel> Pointer;
    using typename Superclass::VectorType;
    using typename Superclass::ParameterVectorType;
    using typename Superclass::StringParameterVectorType;

    PeriodicKernel(T scale, T b, T sigma) : m_Scale(scale), m_B(b), m_Sigma(sigma) { Assign({scale, b, sigma}); }
    PeriodicKernel(const std::string& p1, const std::string& p2, const std::string& p3)
        : PeriodicKernel(this->S2P(p1), this->S2P(p2), this->S2P(p3)) {}

    T operator()(const VectorType& x, const VectorType& y) const override {
        T sum = 0;
        for (std::size_t i = 0; i < x.size(); i++) {
            const double f = std::sin(m_B * (x[i] - y[i]));
            sum += f * f;
        }
        return m_Scale * m_Scale * std::exp(-0.5 * sum / (m_Sigma * m_Sigma));
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        T f1 = 0, f2 = 0;
        for (std::size_t i = 0; i < x.size(); i++) {
            const double r = x[i] - y[i];
            const double sn = std::sin(m_B * r);
            f1 += sn * sn;
            f2 += 2 * r * std::cos(m_B * r) * sn;
        }
        const T s2 = m_Sigma * m_Sigma;
        const T e = std::exp(-0.5 * f1 / s2);
        VectorType D(3);
        D[0] = 2 * m_Scale * e;
        D[1] = -0.5 * m_Scale * m_Scale * e * f2 / s2;
        D[2] = m_Scale * m_Scale * e * f1 / (s2 * m_Sigma);
        return D;
    }
    std::string ToString() const override { return "PeriodicKernel(" + this->ParametersToString(this->m_StringParameters) + ")"; }
    unsigned GetNumberOfParameters() const override { return 3; }
    void SetParameters(const ParameterVectorType& p) override {
        if (p.size() != 3) throw std::string("PeriodicKernel::SetParameters: wrong number of parameters.");
        Assign(p);
    }
    static Pointer Load(const StringParameterVectorType& p) {
        if (p.size() != 3) throw std::string("PeriodicKernel::Load: wrong number of kernel parameters.");
        return Pointer(new PeriodicKernel(Superclass::S2P(p[0]), Superclass::S2P(p[1]), Superclass::S2P(p[2])));
    }
    void Describe(std::vector<gprx_knode>& prog) const override { this->push_leaf(prog, GPRX_K_PERIODIC, this->m_Parameters); }

private:
    void Assign(const ParameterVectorType& p) {
        if (m_Scale == 0) throw std::string("PeriodicKernel: scale parameter has to be positive.");
        if (m_B == 0) throw std::string("PeriodicKernel: period length parameter has to be positive.");
        if (m_Sigma == 0) throw std::string("PeriodicKernel: sigma parameter has to be positive.");
        m_Scale = p[0];
        m_B = p[1];
        m_Sigma = p[2];
        this->m_Parameters = p;
        this->m_StringParameters = {this->P2S(m_Scale), this->P2S(m_B), this->P2S(m_Sigma)};
    }
    T m_Scale, m_B, m_Sigma;
};

// ------------------------------------------------------------------------------------
// Composites: gradient = [k1 params, k2 params]; Product multiplies by the other factor
// (include/Kernel.h:165-178, 314-327).  The string parameters keep the reference layout
// (k1 string twice, both counts, then both parameter lists, include/Kernel.h:264-279).
// ------------------------------------------------------------------------------------
template <class T, bool PRODUCT>
class BinaryKernel : public Kernel<T> {
public:
    typedef Kernel<T> Superclass;
    typedef typename Superclass::Pointer SuperclassPointer;
    using typename Superclass::VectorType;
    using typename Superclass::ParameterVectorType;
    using typename Superclass::StringParameterVectorType;

    BinaryKernel(SuperclassPointer k1, SuperclassPointer k2) : m_Kernel1(k1), m_Kernel2(k2) {
        ParameterVectorType p = k1->GetParameters();
        ParameterVectorType p2 = k2->GetParameters();
        p.insert(p.end(), p2.begin(), p2.end());
        Assign(p);
    }
    T operator()(const VectorType& x, const VectorType& y) const override {
        return PRODUCT ? (*m_Kernel1)(x, y) * (*m_Kernel2)(x, y) : (*m_Kernel1)(x, y) + (*m_Kernel2)(x, y);
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        VectorType D1 = m_Kernel1->GetDerivative(x, y), D2 = m_Kernel2->GetDerivative(x, y);
        const T f1 = PRODUCT ? (*m_Kernel2)(x, y) : T(1);
        const T f2 = PRODUCT ? (*m_Kernel1)(x, y) : T(1);
        VectorType D(D1.size() + D2.size());
        for (std::size_t i = 0; i < D1.size(); i++) D[i] = D1[i] * f1;
        for (std::size_t i = 0; i < D2.size(); i++) D[D1.size() + i] = D2[i] * f2;
        return D;
    }
    std::string ToString() const override {
        return std::string(PRODUCT ? "ProductKernel(" : "SumKernel(") + m_Kernel1->ToString() + "," + m_Kernel2->ToString() + ")";
    }
    unsigned GetNumberOfParameters() const override {
        return m_Kernel1->GetNumberOfParameters() + m_Kernel2->GetNumberOfParameters();
    }
    void SetParameters(const ParameterVectorType& p) override {
        if (p.size() != GetNumberOfParameters())
            throw std::string(PRODUCT ? "ProductKernel::SetParameters: wrong number of parameters."
                                      : "SumKernel::SetParameters: wrong number of parameters.");
        Assign(p);
    }
    const SuperclassPointer GetKernel1() { return m_Kernel1; }
    const SuperclassPointer GetKernel2() { return m_Kernel2; }
    void Describe(std::vector<gprx_knode>& prog) const override {
        m_Kernel1->Describe(prog);
        m_Kernel2->Describe(prog);
        gprx_knode n{};
        n.op = PRODUCT ? GPRX_K_PRODUCT : GPRX_K_SUM;
        prog.push_back(n);
    }

private:
    void Assign(const ParameterVectorType& p) {
        const std::size_t n1 = m_Kernel1->GetNumberOfParameters();
        m_Kernel1->SetParameters(ParameterVectorType(p.begin(), p.begin() + n1));
        m_Kernel2->SetParameters(ParameterVectorType(p.begin() + n1, p.end()));
        this->m_Parameters = p;
        auto& sp = this->m_StringParameters;
        sp.clear();
        sp.push_back(m_Kernel1->ToString());
        sp.push_back(m_Kernel1->ToString());
        const auto s1 = m_Kernel1->GetStringParameters(), s2 = m_Kernel2->GetStringParameters();
        sp.push_back(this->P2S((T)n1));
        sp.push_back(this->P2S((T)(p.size() - n1)));
        sp.insert(sp.end(), s1.begin(), s1.end());
        sp.insert(sp.end(), s2.begin(), s2.end());
    }
    SuperclassPointer m_Kernel1, m_Kernel2;
};

template <class T>
class SumKernel : public BinaryKernel<T, false> {
public:
    typedef std::shared_ptr<SumKernel> Pointer;
    SumKernel(typename Kernel<T>::Pointer k1, typename Kernel<T>::Pointer k2) : BinaryKernel<T, false>(k1, k2) {}
};

template <class T>
class ProductKernel : public BinaryKernel<T, true> {
public:
    typedef std::shared_ptr<ProductKernel> Pointer;
    ProductKernel(typename Kernel<T>::Pointer k1, typename Kernel<T>::Pointer k2) : BinaryKernel<T, true>(k1, k2) {}
};

// ------------------------------------------------------------------------------------
// KernelFactory<T>::GetKernel (include/KernelFactory.h:83-178): recursive parse of the
// ToString() form; the string argument is consumed by reference exactly like the reference.
// ------------------------------------------------------------------------------------
template <class T>
class KernelFactory {
public:
    typedef typename Kernel<T>::Pointer KernelTypePointer;

    static KernelTypePointer GetKernel(std::string& s) {
        const std::size_t open = s.find('(');
        if (open == std::string::npos) throw std::string("KernelFactory::GetKernel: failed to tokanize kernel name string");
        const std::string type = s.substr(0, open);
        if (type == "SumKernel" || type == "ProductKernel") {
            s = s.substr(open + 1);
            KernelTypePointer k1 = GetKernel(s);
            const std::size_t pos = s.find("),");
            if (pos == std::string::npos)
                throw std::string("KernelFactory::GetKernel: failed to tokanize  " +
                                  std::string(type == "SumKernel" ? "sum" : "product") + " kernel name string");
            s = s.substr(pos + 2);
            KernelTypePointer k2 = GetKernel(s);
            if (type == "SumKernel") return KernelTypePointer(new SumKernel<T>(k1, k2));
            return KernelTypePointer(new ProductKernel<T>(k1, k2));
        }
        std::vector<std::string> params;
        std::istringstream rest(s.substr(open + 1));
        std::string tok;
        while (std::getline(rest, tok, ',')) {
            if (tok.find(')') != std::string::npos) break;
            params.push_back(tok);
        }
        if (type == "GaussianKernel") return GaussianKernel<T>::Load(params);
        if (type == "GaussianExpKernel") return GaussianExpKernel<T>::Load(params);
        if (type == "PeriodicKernel") return PeriodicKernel<T>::Load(params);
        if (type == "RationalQuadraticKernel") return RationalQuadraticKernel<T>::Load(params);
        if (type == "WhiteKernel") return WhiteKernel<T>::Load(params);
        throw std::string("KernelFactory::GetKernel: failed to load kernel.");
    }
};

}  // namespace gpr
