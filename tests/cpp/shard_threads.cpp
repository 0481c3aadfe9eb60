// Two ranks as two threads on one GPU, each with its own handle, sharding the
// apply through the C ABI's one-call entry point (mas_shard_apply_device)
// with a host-staged allgather hook -- the shape of a C++ simulator that
// shards without Python.  The union of the ranks' own z entries must equal
// the unsharded mas_apply_device bitwise.  Inputs come from binary files
// written by tests/test_gpu_shard_cpp.py.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "mas_capi.h"

template <class T>
static std::vector<T> load(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    size_t n = f.tellg();
    f.seekg(0);
    std::vector<T> v(n / sizeof(T));
    f.read(reinterpret_cast<char*>(v.data()), n);
    return v;
}

#define CHECK(x)                                                              \
    do {                                                                      \
        int _rc = (x);                                                        \
        if (_rc) {                                                            \
            std::fprintf(stderr, "%s:%d %s -> %d\n", __FILE__, __LINE__, #x, _rc); \
            std::exit(1);                                                     \
        }                                                                     \
    } while (0)

// In-process allgather: every rank deposits its segment in a host buffer,
// waits for the others, then uploads the whole buffer on the given stream.
struct Exchange {
    std::mutex m;
    std::condition_variable cv;
    int world = 0, arrived = 0, generation = 0;
    std::vector<char> buf;
    void barrier() {
        std::unique_lock<std::mutex> lk(m);
        const int gen = generation;
        if (++arrived == world) {
            arrived = 0;
            ++generation;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return generation != gen; });
        }
    }
};
struct RankCtx {
    Exchange* ex;
    int rank;
    int calls = 0;
};

static int host_allgather(const void* send, void* recv, size_t bytes, void* stream, void* user) {
    RankCtx* c = static_cast<RankCtx*>(user);
    Exchange* ex = c->ex;
    hipStream_t s = static_cast<hipStream_t>(stream);
    {
        std::lock_guard<std::mutex> lk(ex->m);
        if (ex->buf.size() < bytes * ex->world) ex->buf.resize(bytes * ex->world);
    }
    ex->barrier();
    if (hipStreamSynchronize(s) != hipSuccess) return 1;  // the restrict is done
    if (hipMemcpy(ex->buf.data() + c->rank * bytes, send, bytes, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    ex->barrier();
    if (hipMemcpyAsync(recv, ex->buf.data(), bytes * ex->world, hipMemcpyHostToDevice, s) != hipSuccess) return 3;
    if (hipStreamSynchronize(s) != hipSuccess) return 4;
    ex->barrier();  // nobody refills buf before every rank has uploaded it
    ++c->calls;
    return 0;
}

struct Inputs {
    std::vector<float> pos, diag, off, r;
    std::vector<int> starts, idx;
    int nV;
};

static mas_handle make_handle(const Inputs& in) {
    mas_config cfg{};
    cfg.device = 0;
    cfg.max_levels = 4;
    mas_handle h = nullptr;
    CHECK(mas_create(&h, &cfg));
    CHECK(mas_allocate(h, in.nV, 0, 0, in.pos.data(), in.starts.data(), in.idx.data(), nullptr, nullptr));
    CHECK(mas_prepare(h, in.diag.data(), in.off.data(), in.starts.data(), nullptr, nullptr, nullptr, nullptr, nullptr,
                      nullptr));
    return h;
}

int main(int argc, char** argv) {
    if (argc < 3) return 2;
    const std::string d = argv[1];
    const int world = std::atoi(argv[2]);
    Inputs in;
    in.pos = load<float>(d + "/pos.bin");
    in.starts = load<int>(d + "/starts.bin");
    in.idx = load<int>(d + "/idx.bin");
    in.diag = load<float>(d + "/diag.bin");
    in.off = load<float>(d + "/off.bin");
    in.r = load<float>(d + "/r.bin");
    in.nV = (int)in.pos.size() / 4;
    const size_t vb = (size_t)in.nV * 16;
    hipSetDevice(0);
    // unsharded reference
    mas_handle h0 = make_handle(in);
    float *dr = nullptr, *dz = nullptr;
    CHECK(hipMalloc(&dr, vb));
    CHECK(hipMalloc(&dz, vb));
    CHECK(hipMemcpy(dr, in.r.data(), vb, hipMemcpyHostToDevice));
    CHECK(mas_apply_device(h0, dz, dr, nullptr));
    CHECK(hipDeviceSynchronize());
    std::vector<float> zref(4 * (size_t)in.nV), zsh(4 * (size_t)in.nV, -12345.f);
    CHECK(hipMemcpy(zref.data(), dz, vb, hipMemcpyDeviceToHost));
    std::vector<int> s2o(in.nV);
    CHECK(mas_get_maps(h0, nullptr, s2o.data(), nullptr, nullptr, nullptr, nullptr, nullptr));

    Exchange ex;
    ex.world = world;
    std::vector<RankCtx> ctx(world);
    std::vector<std::thread> th;
    std::mutex outM;
    int failures = 0;
    for (int g = 0; g < world; ++g) {
        ctx[g] = RankCtx{&ex, g};
        th.emplace_back([&, g] {
            hipSetDevice(0);
            mas_handle h = make_handle(in);
            float *r = nullptr, *z = nullptr;
            CHECK(hipMalloc(&r, vb));
            CHECK(hipMalloc(&z, vb));
            CHECK(hipMemcpy(r, in.r.data(), vb, hipMemcpyHostToDevice));
            CHECK(hipMemset(z, 0xff, vb));
            hipStream_t s;
            CHECK(hipStreamCreate(&s));
            for (int k = 0; k < 3; ++k) {
                const int rc = mas_shard_apply_device(h, g, world, host_allgather, &ctx[g], z, r, s);
                if (rc) {
                    std::lock_guard<std::mutex> lk(outM);
                    std::fprintf(stderr, "rank %d: %d %s\n", g, rc, mas_last_error(h));
                    ++failures;
                    return;
                }
            }
            CHECK(hipStreamSynchronize(s));
            mas_shard sh;
            CHECK(mas_shard_setup(h, g, world, &sh));
            std::vector<float> zl(4 * (size_t)in.nV);
            CHECK(hipMemcpy(zl.data(), z, vb, hipMemcpyDeviceToHost));
            {
                std::lock_guard<std::mutex> lk(outM);
                for (int v = sh.vert_begin; v < sh.vert_end; ++v)
                    std::memcpy(&zsh[4 * (size_t)s2o[v]], &zl[4 * (size_t)s2o[v]], 16);
            }
            hipStreamDestroy(s);
            hipFree(r);
            hipFree(z);
            mas_destroy(h);
        });
    }
    for (auto& t : th) t.join();
    if (failures) return 1;
    const bool same = std::memcmp(zsh.data(), zref.data(), vb) == 0;
    std::printf("world %d hook_calls %d %s\n", world, ctx[0].calls, same ? "BITWISE_EQUAL" : "DIFFERENT");
    mas_destroy(h0);
    return same ? 0 : 1;
}
