// A caller written against the reference surface (SeSchwarzPreconditioner.h:37-178):
// Allocate -> Prepare -> Preconditioning inside a PCG loop, exactly as a
// simulator that uses the reference would call it.  Inputs come from binary
// files written by tests/test_gpu_facade.py; z of the first apply and the PCG
// iteration count are written back for comparison with the oracle.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "SeSchwarzPreconditioner.h"

using namespace SE;

template <class T>
static std::vector<T> load(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    size_t n = f.tellg();
    f.seekg(0);
    std::vector<T> v(n / sizeof(T));
    f.read(reinterpret_cast<char*>(v.data()), n);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    const std::string d = argv[1];
    auto pos = load<SeVec3fSimd>(d + "/pos.bin");
    auto starts = load<int>(d + "/starts.bin");
    auto idx = load<int>(d + "/idx.bin");
    auto diag = load<SeMatrix3f>(d + "/diag.bin");
    auto off = load<SeMatrix3f>(d + "/off.bin");
    auto r0 = load<SeVec3fSimd>(d + "/r.bin");
    const int nV = (int)pos.size();

    SeCsr<int> csr(starts, idx, {});
    SeSchwarzPreconditioner P;
    P.m_positions = pos.data();
    P.m_neighbours = &csr;
    P.AllocatePrecoditioner(nV, 0, 0);
    std::printf("stage allocate\n");
    std::fflush(stdout);
    std::vector<unsigned> efC(1, 0), eeC(1, 0), vfC(nV + 1, 0);
    P.PreparePreconditioner(diag.data(), off.data(), starts.data(), nullptr, nullptr, nullptr, efC.data(), eeC.data(),
                            vfC.data());
    std::vector<SeVec3fSimd> z(nV);
    P.Preconditioning(z.data(), r0.data(), 3 * nV);
    std::printf("stage first_apply\n");
    std::fflush(stdout);
    std::ofstream(d + "/z.bin", std::ios::binary).write(reinterpret_cast<const char*>(z.data()), z.size() * 16);
    // the host-pointer path again: a second apply, a second Prepare through
    // the same arrays, another output array
    {
        std::vector<SeVec3fSimd> z2(nV), z3(nV);
        P.Preconditioning(z2.data(), r0.data(), 3 * nV);
        std::printf("stage second_apply\n");
        std::fflush(stdout);
        P.PreparePreconditioner(diag.data(), off.data(), starts.data(), nullptr, nullptr, nullptr, efC.data(),
                                eeC.data(), vfC.data());
        std::printf("stage second_prepare\n");
        std::fflush(stdout);
        P.Preconditioning(z3.data(), r0.data(), 3 * nV);
        const bool same = std::memcmp(z.data(), z2.data(), z.size() * 16) == 0 &&
                          std::memcmp(z.data(), z3.data(), z.size() * 16) == 0;
        std::printf("host_repeat_bitwise %d\n", same ? 1 : 0);
    }

    // PCG (float64 vectors, fp32 preconditioner) on H x = r0
    auto matvec = [&](const std::vector<double>& x, std::vector<double>& y) {
        for (int v = 0; v < nV; ++v) {
            double acc[3] = {0, 0, 0};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) acc[i] += diag[v](i, j) * x[3 * v + j];
            for (int k = starts[v]; k < starts[v + 1]; ++k) {
                const int u = idx[k];
                for (int i = 0; i < 3; ++i)
                    for (int j = 0; j < 3; ++j) acc[i] += off[k](i, j) * x[3 * u + j];
            }
            for (int i = 0; i < 3; ++i) y[3 * v + i] = acc[i];
        }
    };
    std::vector<SeVec3fSimd> rs(nV), zs(nV);
    auto precond = [&](const std::vector<double>& r, std::vector<double>& zz) {
        for (int v = 0; v < nV; ++v) rs[v] = SeVec3fSimd((float)r[3 * v], (float)r[3 * v + 1], (float)r[3 * v + 2]);
        P.Preconditioning(zs.data(), rs.data(), 3 * nV);
        for (int v = 0; v < nV; ++v)
            for (int i = 0; i < 3; ++i) zz[3 * v + i] = zs[v][i];
    };
    const int n = 3 * nV;
    std::vector<double> x(n, 0), r(n), zz(n), p(n), Ap(n);
    for (int v = 0; v < nV; ++v)
        for (int i = 0; i < 3; ++i) r[3 * v + i] = r0[v][i];
    double nb = 0;
    for (double t : r) nb += t * t;
    nb = std::sqrt(nb);
    precond(r, zz);
    p = zz;
    double rz = 0;
    for (int i = 0; i < n; ++i) rz += r[i] * zz[i];
    int it = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (it = 1; it <= 3000; ++it) {
        if (it % 25 == 0) {
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            std::printf("stage pcg %d %.1f ms\n", it, ms);
            std::fflush(stdout);
        }
        matvec(p, Ap);
        double pAp = 0;
        for (int i = 0; i < n; ++i) pAp += p[i] * Ap[i];
        const double a = rz / pAp;
        double nr = 0;
        for (int i = 0; i < n; ++i) {
            x[i] += a * p[i];
            r[i] -= a * Ap[i];
            nr += r[i] * r[i];
        }
        if (std::sqrt(nr) / nb < 1e-5) break;
        precond(r, zz);
        double rzn = 0;
        for (int i = 0; i < n; ++i) rzn += r[i] * zz[i];
        for (int i = 0; i < n; ++i) p[i] = zz[i] + (rzn / rz) * p[i];
        rz = rzn;
    }
    std::printf("pcg_iterations %d\n", it);
    return 0;
}
