// gp_host_test.cpp — the reference's GaussianProcessTest / IOTest scenarios
// (tests/GaussianProcessTest.cpp:26-330, tests/IOTest.cpp:30-200) restated against the
// gpr:: host API, which runs every fit / predict on the GPU through libgprx.  Same
// inputs, same pass thresholds.  Prints one line per case; exit status = #failures.
// Built by `make cpptests`; driven by tests/test_host_api.py (-m gpu).
#include <cmath>
#include <cstdio>
#include <functional>
#include <iostream>
#include <sstream>
#include <thread>
#include <vector>

#include "gpr/GaussianProcess.h"
#include "gpr/Kernel.h"
#include "gpr/Likelihood.h"
#include "gpr/MatrixIO.h"
#include "gpr/SparseGaussianProcess.h"
#include "gpr/SparseLikelihood.h"
#include "gpr/GaussianProcessInference.h"

using namespace gpr;

template <class T>
using GP = GaussianProcess<T>;

static int g_fail = 0;
static void run(const char* name, const std::function<void()>& f) {
    try {
        f();
        std::printf("PASS %s\n", name);
    } catch (const std::string& s) {
        std::printf("FAIL %s: %s\n", name, s.c_str());
        g_fail++;
    }
    std::fflush(stdout);
}

static void check(bool ok, const std::string& what) {
    if (!ok) throw what;
}
static std::string num(double v) {
    std::ostringstream s;
    s << v;
    return s.str();
}

// GaussianProcessTest Test1: sinus regression, threshold 0.0008
static void gp_test1() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(2.889));
    gp->SetSigma(0);
    const unsigned ns = 10;
    for (unsigned i = 0; i < ns; i++) {
        G::VectorType x(1), y(1);
        x(0) = i * 2 * M_PI / ns;
        y(0) = std::sin(x(0));
        gp->AddSample(x, y);
    }
    gp->Initialize();
    double err = 0;
    for (unsigned i = 0; i < 50; i++) {
        G::VectorType x(1);
        x(0) = i * 2 * M_PI / 50;
        err += std::fabs(gp->Predict(x)(0) - std::sin(x(0)));
    }
    check(err <= 0.0008, num(err));
}

// Test2: 2-D input, sin/cos output, threshold 0.005
static void gp_test2() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(3.24));
    gp->SetSigma(0);
    const unsigned ns = 10;
    for (unsigned i = 0; i < ns; i++) {
        G::VectorType x(2), y(2);
        x(0) = x(1) = i * 2 * M_PI / ns;
        y(0) = std::sin(x(0));
        y(1) = std::cos(x(1));
        gp->AddSample(x, y);
    }
    gp->Initialize();
    double err = 0;
    for (unsigned i = 0; i < 50; i++) {
        G::VectorType x(2);
        x(0) = x(1) = i * 2 * M_PI / 50;
        G::VectorType p = gp->Predict(x);
        err += std::fabs(p(0) - std::sin(x(0))) + std::fabs(p(1) - std::cos(x(1)));
    }
    check(err <= 0.005, num(err));
}

// Test3: 2500 random 73-D samples / labels, sigma 0.01 (a timing case in the reference)
static void gp_test3() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(4));
    gp->SetSigma(0.01);
    for (unsigned i = 0; i < 2500; i++) gp->AddSample(G::VectorType::Random(73), G::VectorType::Random(73));
    gp->Initialize();
    for (unsigned i = 0; i < 50; i++) {
        G::VectorType p = gp->Predict(G::VectorType::Random(73));
        for (std::size_t c = 0; c < p.size(); c++) check(std::isfinite(p(c)), "non-finite prediction");
    }
}

// Test4: four 2-D landmarks, scalar output (the reference only checks it runs)
static void gp_test4() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(3.24));
    gp->SetSigma(0);
    const double pts[4][3] = {{0, 0, 10}, {5, 0, 3}, {5, 8, 3}, {3, 5, 5}};
    for (auto& p : pts) {
        G::VectorType x(2), y(1);
        x(0) = p[0];
        x(1) = p[1];
        y(0) = p[2];
        gp->AddSample(x, y);
    }
    gp->Initialize();
    for (unsigned i = 0; i < 50; i++)
        for (unsigned j = 0; j < 50; j++) {
            G::VectorType x(2);
            x(0) = double(i) / 8;
            x(1) = double(j) / 8;
            check(std::isfinite(gp->Predict(x)(0)), "non-finite prediction");
        }
    // the GP interpolates its landmarks (sigma = 0)
    for (auto& p : pts) {
        G::VectorType x(2);
        x(0) = p[0];
        x(1) = p[1];
        check(std::fabs(gp->Predict(x)(0) - p[2]) < 1e-6, "landmark not interpolated");
    }
}

// Test5: derivative process of a sinus is a cosinus, threshold 0.6
static void gp_test5() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(1));
    gp->SetSigma(0);
    const unsigned ns = 20;
    for (unsigned i = 0; i < ns; i++) {
        G::VectorType x(1), y(1);
        x(0) = i * 4 * M_PI / ns;
        y(0) = std::sin(x(0));
        gp->AddSample(x, y);
    }
    gp->Initialize();
    double err = 0;
    for (unsigned i = 0; i < 50; i++) {
        G::VectorType x(1);
        x(0) = i * 4 * M_PI / 50;
        G::MatrixType D;
        gp->PredictDerivative(x, D);
        err += std::fabs(D(0, 0) - std::cos(x(0)));
    }
    check(err <= 0.6, num(err));
}

// Test6: derivative of a vector-valued process (the reference prints the error only)
static void gp_test6() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(1.2));
    gp->SetSigma(0.01);
    const unsigned ns = 20;
    for (unsigned i = 0; i < ns; i++) {
        G::VectorType x(2), y(3);
        x(0) = x(1) = i * 4 * M_PI / ns;
        y(0) = std::sin(x(0));
        y(1) = std::cos(x(1));
        y(2) = x(0);
        gp->AddSample(x, y);
    }
    gp->Initialize();
    double err = 0;
    for (unsigned i = 0; i < 50; i++) {
        G::VectorType x(2);
        x(0) = x(1) = i * 4 * M_PI / 50;
        G::MatrixType D;
        gp->PredictDerivative(x, D);
        check(D.rows() == 2 && D.cols() == 3, "derivative shape");
        err += std::fabs(D(0, 0) - std::cos(x(0))) + std::fabs(D(1, 0) - std::sin(x(1))) + std::fabs(D(2, 0) - 0.5);
    }
    check(std::isfinite(err), "non-finite derivative");
}

// Test7: a zero Gaussian sigma must throw on evaluation
static void gp_test7() {
    bool threw = false;
    try {
        GaussianKernel<double> k(0);
        GP<double>::VectorType x(1), y(1);
        x(0) = 3.4;
        y(0) = 2.8;
        (void)k(x, y);
    } catch (...) {
        threw = true;
    }
    check(threw, "zero sigma accepted");
}

// IOTest Test1: write / read random matrices (double and float) bit-exactly
static void io_test1() {
    GP<double>::MatrixType a = GP<double>::MatrixType::Random(100, 50);
    WriteMatrix(a, "/tmp/gpr_amd_io_dp.txt");
    auto ar = ReadMatrix<GP<double>::MatrixType>("/tmp/gpr_amd_io_dp.txt");
    GP<float>::MatrixType b = GP<float>::MatrixType::Random(50, 100);
    WriteMatrix(b, "/tmp/gpr_amd_io_sp.txt");
    auto br = ReadMatrix<GP<float>::MatrixType>("/tmp/gpr_amd_io_sp.txt");
    check((a - ar).norm() == 0 && (b - br).norm() == 0, "matrix io mismatch");
}

static std::shared_ptr<GP<float>> io_gp(bool efficient) {
    auto gp = std::make_shared<GP<float>>(std::make_shared<GaussianKernel<float>>(std::sqrt(2)));
    gp->SetSigma(0);
    if (efficient) gp->SetEfficientStorage(true);
    for (unsigned i = 0; i < 10; i++) {
        GP<float>::VectorType x(2), y(2);
        x(0) = x(1) = i * 2 * M_PI / 10;
        y(0) = std::sin(x(0));
        y(1) = std::cos(x(1));
        gp->AddSample(x, y);
    }
    gp->Initialize();
    return gp;
}

// IOTest Test2: save / load round trip compares equal
static void io_test2() {
    auto gp = io_gp(false);
    gp->Save("/tmp/gpr_amd_io_test-");
    auto rd = std::make_shared<GP<float>>(std::make_shared<GaussianKernel<float>>(1));
    rd->Load("/tmp/gpr_amd_io_test-");
    check(*gp == *rd, "read/write");
}

// IOTest Test3.1 / 3.2: efficient storage, late core construction changes ==
static void io_test3() {
    auto gp0 = std::make_shared<GP<float>>(std::make_shared<GaussianKernel<float>>(1));
    check(!gp0->GetEfficientStorage(), "efficient storage must be off by default");
    auto gp = io_gp(true);
    GP<float>::VectorType x(2);
    x(0) = x(1) = 2.56 * 2 * M_PI / 10;
    GP<float>::VectorType yt = gp->Predict(x);
    gp->Save("/tmp/gpr_amd_io_test-");
    {
        auto rd = std::make_shared<GP<float>>(std::make_shared<GaussianKernel<float>>(1));
        rd->Load("/tmp/gpr_amd_io_test-");
        check(*gp == *rd, "3.1 compare");
        check((yt - rd->Predict(x)).norm() < 1e-6, "3.1 predict " + num((yt - rd->Predict(x)).norm()));
    }
    {
        auto rd = std::make_shared<GP<float>>(std::make_shared<GaussianKernel<float>>(1));
        rd->Load("/tmp/gpr_amd_io_test-");
        (void)(*rd)(x, x);
        check(!(*gp == *rd), "Comparison with late core matrix construction not right.");
        (void)(*gp)(x, x);
        check(*gp == *rd, "Comparison with late core matrix construction not right.");
        check((yt - rd->Predict(x)).norm() < 1e-6, "3.2 predict");
    }
}

// Load into a GP that was already fitted on OTHER samples (a different count, both ways): the
// device must drop the old samples, factor and alpha, and predict / operator() must then match
// the GP that was saved (the reference's Load replaces every member, lib/GaussianProcess.cpp
// :184-268).
static std::shared_ptr<GP<double>> reload_gp(unsigned n, double phase) {
    auto gp = std::make_shared<GP<double>>(std::make_shared<GaussianKernel<double>>(0.7, 1.3));
    gp->SetSigma(0.05);
    for (unsigned i = 0; i < n; i++) {
        GP<double>::VectorType x(2), y(1);
        x(0) = i * 6.0 / n;
        x(1) = std::cos(0.3 * i + phase);
        y(0) = std::sin(x(0) + phase) + 0.3 * x(1);
        gp->AddSample(x, y);
    }
    gp->Initialize();
    return gp;
}

static void io_reload_test() {
    for (int dir = 0; dir < 2; dir++) {
        const unsigned ns = dir ? 61 : 23, nt = dir ? 23 : 61;  // saved size, target's own size
        auto src = reload_gp(ns, 0.4);
        src->Save("/tmp/gpr_amd_reload_test-");
        auto dst = reload_gp(nt, 1.9);
        GP<double>::VectorType x(2);
        x(0) = 2.2;
        x(1) = 0.1;
        (void)dst->Predict(x);
        (void)(*dst)(x, x);  // the target holds its own factor and alpha on the device
        dst->Load("/tmp/gpr_amd_reload_test-");
        for (int q = 0; q < 5; q++) {
            x(0) = 0.3 + 1.1 * q;
            x(1) = 0.2 * q - 0.4;
            const double a = src->Predict(x)(0), b = dst->Predict(x)(0);
            check(std::fabs(a - b) <= 1e-9 * std::max(1.0, std::fabs(a)), "predict after Load " + num(a) + " vs " + num(b));
            const double ca = (*src)(x, x), cb = (*dst)(x, x);
            check(std::fabs(ca - cb) <= 1e-9, "posterior variance after Load " + num(ca) + " vs " + num(cb));
        }
    }
}

// Likelihood: value and gradient through the host classes are finite and the gradient
// matches a central difference of the value (GaussianLikelihoodTest's consistency idea).
static void lik_test() {
    typedef GP<double> G;
    auto k = std::make_shared<GaussianKernel<double>>(1.3, 0.8);
    auto gp = std::make_shared<G>(k);
    gp->SetSigma(0.1);
    for (unsigned i = 0; i < 64; i++) {
        G::VectorType x(1), y(1);
        x(0) = -3 + 6.0 * i / 63;
        y(0) = std::sin(2 * x(0)) + 0.1 * std::cos(7 * x(0));
        gp->AddSample(x, y);
    }
    GaussianLogLikelihood<double> lik;
    auto vg = lik.GetValueAndParameterDerivatives(gp);
    check(std::isfinite(vg.first(0)), "likelihood not finite");
    auto p = k->GetParameters();
    for (std::size_t i = 0; i < p.size(); i++) {
        const double h = 1e-5;
        auto pp = p, pm = p;
        pp[i] += h;
        pm[i] -= h;
        k->SetParameters(pp);
        gp->SetKernel(k);
        const double vp = lik(gp)(0);
        k->SetParameters(pm);
        gp->SetKernel(k);
        const double vm = lik(gp)(0);
        const double fd = (vp - vm) / (2 * h);
        check(std::fabs(fd - vg.second(i)) <= 1e-4 * std::max(1.0, std::fabs(fd)),
              "grad " + num(vg.second(i)) + " vs fd " + num(fd));
    }
    k->SetParameters(p);
    GaussianLikelihood<double> plain;
    const double lv = plain(gp)(0);
    check(std::isfinite(lv) && lv >= 0, "GaussianLikelihood value " + num(lv));
}

// SparseGaussianProcess: dense sinus samples, every 10th as an inducing point
// (the regression setting of tests/SparseInferenceTest.cpp), predictions close to sin.
static void sparse_test() {
    typedef SparseGaussianProcess<double> S;
    auto gp = std::make_shared<S>(std::make_shared<GaussianKernel<double>>(0.8), 1e-6);
    gp->SetSigma(0.01);
    for (unsigned i = 0; i < 400; i++) {
        S::VectorType x(1), y(1);
        x(0) = i * 2 * M_PI / 400;
        y(0) = std::sin(x(0));
        gp->AddSample(x, y);
        if (i % 10 == 0) gp->AddInducingSample(x, y);
    }
    gp->Initialize();
    check(gp->GetNumberOfInducingSamples() == 40, "inducing count");
    double err = 0;
    for (unsigned i = 0; i < 50; i++) {
        S::VectorType x(1);
        x(0) = 0.1 + i * 6.0 / 50;
        err += std::fabs(gp->Predict(x)(0) - std::sin(x(0)));
        const double v = (*gp)(x, x);
        check(std::isfinite(v) && v > -1e-6, "sparse posterior variance " + num(v));
    }
    check(err < 0.05, "sparse predict error " + num(err));
}

// SparseGaussianLogLikelihood (include/SparseLikelihood.h:231-344): value and gradient on a
// sparse GP (every 8th dense sample inducing) vs central differences of the value; operator(),
// GetValueAndParameterDerivatives and GetValueAndJacobian agree; a dense GP is rejected with
// the reference's cast message.
static void sparse_lik_test() {
    typedef SparseGaussianProcess<double> S;
    auto k = std::make_shared<GaussianKernel<double>>(0.9, 1.2);
    auto gp = std::make_shared<S>(k, 1e-3);
    gp->SetSigma(0.2);
    for (unsigned i = 0; i < 320; i++) {
        S::VectorType x(1), y(1);
        x(0) = -3 + 6.0 * i / 319;
        y(0) = std::sin(2 * x(0)) + 0.1 * std::cos(7 * x(0));
        gp->AddSample(x, y);
        if (i % 16 == 0) gp->AddInducingSample(x, y);
    }
    SparseGaussianLogLikelihood<double> lik;
    auto vg = lik.GetValueAndParameterDerivatives(gp);
    check(std::isfinite(vg.first(0)), "sparse likelihood not finite");
    check(lik(gp)(0) == vg.first(0), "operator() vs GetValueAndParameterDerivatives");
    auto vj = lik.GetValueAndJacobian(gp);
    check(vj.second.rows() == 1 && vj.second.cols() == vg.second.size(), "Jacobian shape");
    auto p = k->GetParameters();
    for (std::size_t i = 0; i < p.size(); i++) {
        check(vj.second(0, i) == vg.second(i), "Jacobian row vs gradient");
        // Richardson-extrapolated central differences (cond(Kmm + jitter I) ~ 1e4 limits plain
        // differences at small steps to ~1e-4)
        auto cd = [&](double h) {
            auto pp = p, pm = p;
            pp[i] += h;
            pm[i] -= h;
            k->SetParameters(pp);
            const double vp = lik(gp)(0);
            k->SetParameters(pm);
            const double vm = lik(gp)(0);
            return (vp - vm) / (2 * h);
        };
        const double fd = (4 * cd(5e-4) - cd(1e-3)) / 3;
        check(std::fabs(fd - vg.second(i)) <= 1e-4 * std::max(1.0, std::fabs(fd)),
              "sparse grad " + num(vg.second(i)) + " vs fd " + num(fd));
    }
    k->SetParameters(p);
    auto dense = std::make_shared<GP<double>>(k);
    bool threw = false;
    try {
        lik(dense);
    } catch (std::string& e) {
        threw = e == "SparseGaussianLogLikelihood: cannot cast to SparseGaussianProcess";
    }
    check(threw, "dense GP must be rejected");
}

// MaximumLikelihoodTest2 Test1 (tests/MaximumLikelihoodTest2.cpp:36-117): GaussianExp kernel
// hyper-parameters by GaussianProcessInference::Optimize (100 Gauss-Newton steps of 0.1) on
// 200 noisy samples of (0.5 sin(11x) + sin(4x)) x^2, then the exp'd parameters in a Gaussian
// kernel; mean absolute prediction error over 1000 points <= 2 (the reference's bar).  The
// reference draws its noise from boost's normal_distribution seeded with time(0); here a fixed
// LCG + Box-Muller (sd 0.1).
static void ml_test1() {
    typedef GP<double> G;
    const unsigned n = 200;
    const double noise = 0.1;
    auto f = [](double x) { return (0.5 * std::sin(x + 10 * x) + std::sin(4 * x)) * x * x; };
    unsigned long long st = 0x9E3779B97F4A7C15ull;
    auto unif = [&]() {
        st = st * 6364136223846793005ull + 1442695040888963407ull;
        return ((st >> 11) + 0.5) * (1.0 / 9007199254740992.0);
    };
    const double start = -5, stop = 10;
    auto gk = std::make_shared<GaussianExpKernel<double>>(1, 1);
    auto gp = std::make_shared<G>(gk);
    gp->SetSigma(noise);
    for (unsigned i = 0; i < n; i++) {
        const double x = start + i * (stop - start) / n;
        const double r = noise * std::sqrt(-2 * std::log(unif())) * std::cos(2 * M_PI * unif());
        G::VectorType xv(1), yv(1);
        xv(0) = x;
        yv(0) = f(x) + r;
        gp->AddSample(xv, yv);
    }
    auto lh = std::make_shared<GaussianLogLikelihood<double>>();
    GaussianProcessInference<double> gpi(lh, gp, 1e-1, 100);
    gpi.Optimize(false, true);
    auto parameters = gpi.GetParameters();
    for (auto& p : parameters) p = std::exp(p);
    auto k = std::make_shared<GaussianKernel<double>>(1, 1);
    k->SetParameters(parameters);
    gp->SetKernel(k);
    double error = 0;
    const unsigned gt_n = 1000;
    for (unsigned i = 0; i < gt_n; i++) {
        const double x = start + i * (stop - start) / gt_n;
        G::VectorType xv(1);
        xv(0) = x;
        error += std::fabs(gp->Predict(xv)(0) - f(x));
    }
    check(error / gt_n <= 2, "ML Test1 mean error " + num(error / gt_n));
}

// SparseInferenceTest-style loop: Optimize2 (Gauss-Newton on J^T J) of a sparse GP's kernel
// parameters with SparseGaussianLogLikelihood; the likelihood must not decrease.
static void sparse_ml_test() {
    typedef SparseGaussianProcess<double> S;
    auto k = std::make_shared<GaussianKernel<double>>(2.0, 1.0);
    auto gp = std::make_shared<S>(k, 1e-3);
    gp->SetSigma(0.1);
    for (unsigned i = 0; i < 400; i++) {
        S::VectorType x(1), y(1);
        x(0) = -3 + 6.0 * i / 399;
        y(0) = std::sin(2 * x(0));
        gp->AddSample(x, y);
        if (i % 16 == 0) gp->AddInducingSample(x, y);
    }
    auto lh = std::make_shared<SparseGaussianLogLikelihood<double>>();
    const double v0 = (*lh)(gp)(0);
    GaussianProcessInference<double> gpi(lh, gp, 1e-2, 20);
    gpi.Optimize2(false, false);
    k->SetParameters(gpi.GetParameters());
    const double v1 = (*lh)(gp)(0);
    check(std::isfinite(v1) && v1 >= v0, "sparse inference: likelihood " + num(v0) + " -> " + num(v1));
}

// PosteriorProcessTest Test1 (tests/PosteriorProcessTest.cpp:51-95): the credible interval
// is exactly 2 sqrt(gp(x, x)), sigma = 1e-5, 20 sinus samples.
static void posterior_test1() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(0.5));
    gp->SetSigma(0.00001);
    for (unsigned i = 0; i < 20; i++) {
        G::VectorType x(1), y(1);
        x(0) = i * 2 * M_PI / 20;
        y(0) = std::sin(x(0));
        gp->AddSample(x, y);
    }
    gp->Initialize();
    for (unsigned i = 0; i < 50; i++) {
        G::VectorType x(1);
        x(0) = i * 2 * M_PI / 50 * 1.3;
        const double c = 2 * std::sqrt((*gp)(x, x)) - gp->GetCredibleInterval(x);
        check(c == 0, "credible interval not correct at x = " + num(x(0)) + " (gp(x,x) = " + num((*gp)(x, x)) + ")");
    }
}

// PosteriorProcessTest Test2 (tests/PosteriorProcessTest.cpp:97-165): the posterior kernel
// matrix over [0, 5) of a noise-free GP through 4 landmarks, its rows filled by Predict and
// operator() running CONCURRENTLY (the reference's omp parallel for, :120-134; here 8
// std::threads).  The reference then samples the posterior (Eigen eigensolver, absent here)
// and checks every sample equals the mean at the landmarks (|r - mean| <= 1e-9): that holds
// iff the posterior covariance vanishes on the landmark rows, which is checked directly.
// Run on a fresh GP and on one restored by Load, whose factor is rebuilt lazily by the first
// operator() -- the refit that must not race the concurrent Predict calls.
static void posterior_test2_on(GP<double>& gp) {
    typedef GP<double> G;
    const unsigned ns = 50;
    std::vector<double> mean(ns), K(ns * ns, 0.0);
    std::vector<std::string> errs(8);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < 8; t++)
        th.emplace_back([&, t]() {
            try {
                for (unsigned i = t; i < ns; i += 8) {
                    G::VectorType x1(1);
                    x1(0) = i * 5.0 / ns;
                    mean[i] = gp.Predict(x1)(0);
                    for (unsigned j = i; j < ns; j++) {
                        G::VectorType x2(1);
                        x2(0) = j * 5.0 / ns;
                        K[i * ns + j] = K[j * ns + i] = gp(x1, x2);
                    }
                }
            } catch (const std::string& e) {
                errs[t] = e;
            }
        });
    for (auto& x : th) x.join();
    for (auto& e : errs) check(e.empty(), "concurrent call failed: " + e);
    for (unsigned l : {10u, 20u, 30u, 40u}) {
        for (unsigned j = 0; j < ns; j++)
            check(std::fabs(K[l * ns + j]) <= 1e-9, "posterior covariance at landmark " + num(l) + ", " + num(j) +
                                                     " = " + num(K[l * ns + j]));
        const double y = (l == 10) ? 0.0 : (l == 30 ? 0.5 : 1.0);
        check(std::fabs(mean[l] - y) <= 1e-9, "mean at landmark " + num(l) + " = " + num(mean[l]));
    }
    for (unsigned i = 0; i < ns; i++) check(K[i * ns + i] >= -1e-9, "negative posterior variance");
}

static std::shared_ptr<GP<double>> landmark_gp() {
    typedef GP<double> G;
    auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(1));
    gp->SetSigma(0);
    const double xs[4] = {1, 2, 3, 4}, ys[4] = {0, 1, 0.5, 1};
    for (int i = 0; i < 4; i++) {
        G::VectorType x(1), y(1);
        x(0) = xs[i];
        y(0) = ys[i];
        gp->AddSample(x, y);
    }
    gp->Initialize();
    return gp;
}

static void posterior_test2() {
    auto gp = landmark_gp();
    posterior_test2_on(*gp);
}

static void posterior_test2_loaded() {
    auto gp = landmark_gp();
    gp->Save("/tmp/gpr_amd_post_test-");
    auto rd = std::make_shared<GP<double>>(std::make_shared<GaussianKernel<double>>(3));
    rd->Load("/tmp/gpr_amd_post_test-");
    posterior_test2_on(*rd);
}

// A user Kernel<T> subclass without a device form (no Describe override): the GP evaluates
// it through the virtual operator() / GetDerivative, as the reference does for every kernel
// (include/Kernel.h:52-59), and factors / solves / reduces on the device.  Same Gaussian
// function as the built-in kernel: identical predictions, intervals and likelihood.
template <class T>
class UserGaussian : public Kernel<T> {
public:
    typedef typename Kernel<T>::VectorType VectorType;
    typedef typename Kernel<T>::ParameterVectorType ParameterVectorType;
    UserGaussian(T sigma, T scale) : s(sigma), c(scale) {
        this->m_Parameters = {sigma, scale};
        this->m_StringParameters = {this->P2S(sigma), this->P2S(scale)};
    }
    T operator()(const VectorType& x, const VectorType& y) const override {
        const T r = (x - y).norm();
        return c * c * std::exp(-0.5 * r * r / (s * s));
    }
    VectorType GetDerivative(const VectorType& x, const VectorType& y) const override {
        const T r = (x - y).norm(), f = std::exp(-0.5 * r * r / (s * s));
        VectorType D(2);
        D[0] = c * c * r * r / (s * s * s) * f;
        D[1] = 2 * c * f;
        return D;
    }
    std::string ToString() const override { return "UserGaussian(" + this->ParametersToString(this->m_StringParameters) + ")"; }
    unsigned GetNumberOfParameters() const override { return 2; }
    void SetParameters(const ParameterVectorType& p) override {
        s = p[0];
        c = p[1];
        this->m_Parameters = p;
    }

private:
    T s, c;
};

static void host_kernel_test() {
    typedef GP<double> G;
    auto gu = std::make_shared<G>(std::make_shared<UserGaussian<double>>(0.7, 1.3));
    auto gd = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(0.7, 1.3));
    for (auto& gp : {gu, gd}) {
        gp->SetSigma(0.1);
        for (unsigned i = 0; i < 60; i++) {
            G::VectorType x(2), y(1);
            x(0) = std::sin(0.37 * i);
            x(1) = std::cos(1.3 * i);
            y(0) = std::sin(2 * x(0)) + 0.5 * x(1);
            gp->AddSample(x, y);
        }
        gp->Initialize();
    }
    for (unsigned i = 0; i < 20; i++) {
        G::VectorType x(2), x2(2);
        x(0) = 0.05 * i - 0.5;
        x(1) = 0.3 - 0.02 * i;
        x2(0) = x(1);
        x2(1) = x(0);
        G::MatrixType Du, Dd;
        const double mu = gu->PredictDerivative(x, Du)(0), md = gd->PredictDerivative(x, Dd)(0);
        check(std::fabs(mu - md) <= 1e-9 * std::max(1.0, std::fabs(md)), "mean " + num(mu) + " vs " + num(md));
        for (unsigned k = 0; k < 2; k++)
            check(std::fabs(Du(k, 0) - Dd(k, 0)) <= 1e-8 * std::max(1.0, std::fabs(Dd(k, 0))), "derivative");
        const double cu = (*gu)(x, x2), cd = (*gd)(x, x2);
        check(std::fabs(cu - cd) <= 1e-9, "posterior covariance " + num(cu) + " vs " + num(cd));
        check(std::fabs(gu->GetCredibleInterval(x) - gd->GetCredibleInterval(x)) <= 1e-7, "credible interval");
    }
    GaussianLogLikelihood<double> lik;
    auto vu = lik.GetValueAndParameterDerivatives(gu), vd = lik.GetValueAndParameterDerivatives(gd);
    check(std::fabs(vu.first(0) - vd.first(0)) <= 1e-8 * std::fabs(vd.first(0)),
          "likelihood " + num(vu.first(0)) + " vs " + num(vd.first(0)));
    for (unsigned p = 0; p < 2; p++)
        check(std::fabs(vu.second(p) - vd.second(p)) <= 1e-7 * std::max(1.0, std::fabs(vd.second(p))),
              "likelihood gradient " + num(vu.second(p)) + " vs " + num(vd.second(p)));
}

// SetInversionMethod (lib/GaussianProcess.cpp:531-618): the SVD methods' exact inverse and the
// self-adjoint (Cholesky) branch give the default method's regression to rounding.
static void inversion_methods_test() {
    typedef GP<double> G;
    std::vector<std::shared_ptr<G>> gps;
    for (int meth = 0; meth < 4; meth++) {
        auto gp = std::make_shared<G>(std::make_shared<GaussianKernel<double>>(1.1, 0.9));
        gp->SetSigma(0.05);
        gp->SetInversionMethod(static_cast<G::InversionMethod>(meth));
        for (unsigned i = 0; i < 80; i++) {
            G::VectorType x(1), y(1);
            x(0) = i * 0.1;
            y(0) = std::sin(x(0));
            gp->AddSample(x, y);
        }
        gp->Initialize();
        gps.push_back(gp);
    }
    for (unsigned i = 0; i < 30; i++) {
        G::VectorType x(1);
        x(0) = 0.27 * i;
        const double m0 = gps[0]->Predict(x)(0);
        for (int meth = 1; meth < 4; meth++)
            check(std::fabs(gps[meth]->Predict(x)(0) - m0) <= 1e-8, "method " + num(meth) + " prediction");
    }
}

int main() {
    run("GaussianProcessTest1", gp_test1);
    run("GaussianProcessTest2", gp_test2);
    run("GaussianProcessTest3", gp_test3);
    run("GaussianProcessTest4", gp_test4);
    run("GaussianProcessTest5", gp_test5);
    run("GaussianProcessTest6", gp_test6);
    run("GaussianProcessTest7", gp_test7);
    run("IOTest1", io_test1);
    run("IOTest2", io_test2);
    run("IOTest3", io_test3);
    run("IOReloadIntoFittedGP", io_reload_test);
    run("LikelihoodGradient", lik_test);
    run("SparseRegression", sparse_test);
    run("SparseLogLikelihood", sparse_lik_test);
    run("MaximumLikelihoodTest1", ml_test1);
    run("SparseInferenceOptimize2", sparse_ml_test);
    run("PosteriorProcessTest1", posterior_test1);
    run("PosteriorProcessTest2", posterior_test2);
    run("PosteriorProcessTest2Loaded", posterior_test2_loaded);
    run("HostEvaluatedKernel", host_kernel_test);
    run("InversionMethods", inversion_methods_test);
    return g_fail;
}
