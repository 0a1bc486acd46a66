// host_cpu_test.cpp — host-only checks of the gpr:: C++ API (no GPU needed):
// kernel evaluation / derivatives vs central differences (tests/KernelDerivativeTest.cpp
// idea), ToString -> KernelFactory round trips (tests/IOTest.cpp kernel cases), the
// matrix file format, the device lowering (Describe), and that a GaussianProcess fails
// loudly (std::string) when no GPU is visible — there is no CPU fallback.
// Driven by tests/test_host_api.py (not gpu); prints one line per case.
#include <cmath>
#include <cstdio>
#include <functional>
#include <sstream>

#include "gpr/GaussianProcess.h"
#include "gpr/GaussianProcessInference.h"
#include "gpr/Kernel.h"
#include "gpr/MatrixIO.h"

using namespace gpr;
static int g_fail = 0;
static void run(const char* name, const std::function<void()>& f) {
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (const std::string& s) {
        std::printf("FAIL %s: %s\n", name, s.c_str());
        g_fail++;
    }
}
static void check(bool ok, const std::string& what) {
    if (!ok) throw what;
}

typedef Kernel<double>::Pointer KP;
static std::vector<KP> kernels() {
    auto g = std::make_shared<GaussianKernel<double>>(1.7, 0.9);
    auto p = std::make_shared<PeriodicKernel<double>>(0.8, M_PI, 1.3);
    auto r = std::make_shared<RationalQuadraticKernel<double>>(1.1, 0.7, 2.0);
    auto e = std::make_shared<GaussianExpKernel<double>>(1.2, 0.5);
    return {g, p, r, e, std::make_shared<SumKernel<double>>(g, p), std::make_shared<ProductKernel<double>>(r, e),
            std::make_shared<SumKernel<double>>(std::make_shared<ProductKernel<double>>(g, p), r)};
}

// d k / d theta by central differences on the parameter vector
static void deriv_test() {
    Kernel<double>::VectorType x(3), y(3);
    x(0) = 0.3, x(1) = -1.1, x(2) = 0.7;
    y(0) = 1.0, y(1) = 0.2, y(2) = -0.4;
    for (auto k : kernels()) {
        auto p = k->GetParameters();
        auto D = k->GetDerivative(x, y);
        check(D.size() == p.size(), k->ToString() + ": derivative size");
        for (std::size_t i = 0; i < p.size(); i++) {
            const double h = 1e-6;
            auto pp = p, pm = p;
            pp[i] += h;
            pm[i] -= h;
            k->SetParameters(pp);
            const double vp = (*k)(x, y);
            k->SetParameters(pm);
            const double vm = (*k)(x, y);
            k->SetParameters(p);
            const double fd = (vp - vm) / (2 * h);
            if (std::fabs(fd - D[i]) > 1e-5 * std::max(1.0, std::fabs(fd))) {
                std::ostringstream s;
                s << k->ToString() << " param " << i << ": " << D[i] << " vs " << fd;
                throw s.str();
            }
        }
    }
}

static void factory_test() {
    for (auto k : kernels()) {
        std::string s = k->ToString();
        auto k2 = KernelFactory<double>::GetKernel(s);
        check(*k == *k2, "round trip " + k->ToString() + " -> " + k2->ToString());
        std::vector<gprx_knode> a, b;
        k->Describe(a);
        k2->Describe(b);
        check(a.size() == b.size(), "describe size");
        for (std::size_t i = 0; i < a.size(); i++)
            check(a[i].op == b[i].op && a[i].p[0] == b[i].p[0] && a[i].p[1] == b[i].p[1] && a[i].p[2] == b[i].p[2],
                  "describe node");
    }
    bool threw = false;
    try {
        std::string bad = "NoSuchKernel(1,)";
        KernelFactory<double>::GetKernel(bad);
    } catch (const std::string&) {
        threw = true;
    }
    check(threw, "unknown kernel accepted");
}

static void io_test() {
    auto a = DenseMatrix<double>::Random(37, 11);
    WriteMatrix(a, "/tmp/gpr_amd_cpu_io.txt");
    auto b = ReadMatrix<DenseMatrix<double>>("/tmp/gpr_amd_cpu_io.txt");
    check(b.rows() == 37 && b.cols() == 11 && (a - b).norm() == 0, "round trip");
}

static void no_device_test() {
    auto gp = std::make_shared<GaussianProcess<double>>(std::make_shared<GaussianKernel<double>>(1.0));
    GaussianProcess<double>::VectorType x(1), y(1);
    x(0) = 1;
    y(0) = 2;
    gp->AddSample(x, y);
    bool threw = false;
    try {
        gp->Initialize();
    } catch (const std::string&) {
        threw = true;
    }
    check(threw, "Initialize without a GPU must throw");
}

static void dim_test() {
    auto gp = std::make_shared<GaussianProcess<double>>(std::make_shared<GaussianKernel<double>>(1.0));
    GaussianProcess<double>::VectorType x(2), y(1), x3(3);
    gp->AddSample(x, y);
    bool threw = false;
    try {
        gp->AddSample(x3, y);
    } catch (const std::string& s) {
        threw = s.find("GaussianProcess::AddSample: dimension of input vector (3)") == 0;
    }
    check(threw, "dimension mismatch message");
}

// pinv (include/Prior.h:38-55 restated in gpr/GaussianProcessInference.h): Moore-Penrose
// conditions on a full-rank and a rank-deficient matrix, and the rank-1 g g^T of Optimize,
// whose pseudo-inverse times g is g / |g|^2.
static void pinv_test() {
    typedef GaussianProcess<double>::MatrixType MT;
    auto mul = [](const MT& a, const MT& b) {
        MT c(a.rows(), b.cols());
        for (std::size_t i = 0; i < a.rows(); i++)
            for (std::size_t j = 0; j < b.cols(); j++) {
                double s = 0;
                for (std::size_t k = 0; k < a.cols(); k++) s += a(i, k) * b(k, j);
                c(i, j) = s;
            }
        return c;
    };
    auto maxdiff = [](const MT& a, const MT& b) {
        double m = 0;
        for (std::size_t i = 0; i < a.rows(); i++)
            for (std::size_t j = 0; j < a.cols(); j++) m = std::max(m, std::fabs(a(i, j) - b(i, j)));
        return m;
    };
    MT A(5, 5), R(5, 5);
    unsigned st = 12345;
    for (std::size_t i = 0; i < 5; i++)
        for (std::size_t j = 0; j < 5; j++) {
            st = st * 1103515245u + 12345u;
            A(i, j) = ((st >> 8) % 1000) / 500.0 - 1.0;
        }
    for (std::size_t i = 0; i < 5; i++)  // rank 3: rows 3, 4 are combinations of rows 0-2
        for (std::size_t j = 0; j < 5; j++) R(i, j) = i < 3 ? A(i, j) : A(0, j) * (i - 2.0) + A(1, j);
    for (const MT* M : {&A, &R}) {
        const MT P = pinv<MT>(*M);
        check(maxdiff(mul(mul(*M, P), *M), *M) < 1e-12, "pinv: A P A != A");
        check(maxdiff(mul(mul(P, *M), P), P) < 1e-10, "pinv: P A P != P");
    }
    const double g[3] = {0.3, -2.0, 0.7};
    MT G(3, 3);
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) G(a, b) = g[a] * g[b];
    const MT P = pinv<MT>(G);
    const double g2 = 0.09 + 4.0 + 0.49;
    for (int a = 0; a < 3; a++) {
        double u = 0;
        for (int b = 0; b < 3; b++) u += P(a, b) * g[b];
        check(std::fabs(u - g[a] / g2) < 1e-12, "pinv(g g^T) g != g / |g|^2");
    }
}

int main(int argc, char** argv) {
    run("PseudoInverse", pinv_test);
    run("KernelDerivatives", deriv_test);
    run("KernelFactoryRoundTrip", factory_test);
    run("MatrixIO", io_test);
    run("DimensionCheck", dim_test);
    if (argc > 1 && std::string(argv[1]) == "--no-device") run("NoDeviceFailsLoudly", no_device_test);
    return g_fail;
}
