// mas_capi.hip -- C ABI entry points (include/mas_capi.h) and shared helpers.
//
// The handle owns every device buffer; all work is enqueued on one HIP stream.
// Host-pointer entry points stage through device buffers and synchronise, so a
// PCG loop that calls the reference's three methods keeps working unchanged
// (SeSchwarzPreconditioner.h:56-63).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <new>

#include <hipcub/hipcub.hpp>

#include "mas_internal.h"

namespace mas {

static thread_local std::string* tlErrSink = nullptr;
ErrorSink::ErrorSink(std::string* sink) { tlErrSink = sink; }
ErrorSink::~ErrorSink() { tlErrSink = nullptr; }

int fail(mas_context* h, int code, const std::string& msg) {
    if (tlErrSink) *tlErrSink = msg;
    else if (h) h->err = msg;
    return code;
}

int hip_check(mas_context* h, hipError_t e, const char* what) {
    if (e == hipSuccess) return MAS_OK;
    return fail(h, MAS_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

int ensure(mas_context* h, Buffer& b, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (b.bytes >= bytes) return MAS_OK;
    // every allocation of a handle lives on its device: a thread that forgot
    // hipSetDevice (the early-path worker selects it per job) fails loudly here
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != h->device)
        return fail(h, MAS_ERR_STATE, "allocation on device " + std::to_string(dev) + " for a handle of device " +
                                          std::to_string(h->device));
    if (b.p) {
        hipStreamSynchronize(h->stream);
        hipFree(b.p);
        b.p = nullptr;
        b.bytes = 0;
    }
    hipError_t e = hipMalloc(&b.p, bytes);
    if (e != hipSuccess) {
        b.p = nullptr;
        return fail(h, MAS_ERR_NOMEM, std::string("hipMalloc ") + std::to_string(bytes) + " B: " + hipGetErrorString(e));
    }
    b.bytes = bytes;
    return MAS_OK;
}

// Small device -> host reads (sizes the host needs before its next
// launches) through pinned memory: one single-lane kernel copies up to 8 ints
// to the pinned words and then publishes a sequence number; the host spins
// on that word.  hipStreamSynchronize + a pageable copy cost ~40 us of
// wake-up each (7 of them per Prepare); this costs the
// kernel's completion plus a few microseconds.  Falls back to a stream
// synchronisation after 5 s (never spins forever).
struct ReadBackArgs {
    const int* src[8];
    int n;
};
__global__ void k_readback(ReadBackArgs a, int* host, int seq) {
    if (threadIdx.x != 0) return;
    int v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = i < a.n ? *a.src[i] : 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        if (i < a.n) __hip_atomic_store(host + 1 + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(host, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int read_back_post(mas_context* h, hipStream_t s, std::initializer_list<const int*> src, int* seqOut) {
    if (src.size() > 8) return fail(h, MAS_ERR_ARG, "read_back: at most 8 words");
    if (!h->rbHost) {
        void* p = nullptr;
        int rc = hip_check(h, hipHostMalloc(&p, 16 * sizeof(int), hipHostMallocCoherent), "pinned read-back words");
        if (rc) return rc;
        h->rbHost = static_cast<int*>(p);
        std::memset(p, 0, 16 * sizeof(int));
    }
    ReadBackArgs a{};
    a.n = (int)src.size();
    int i = 0;
    for (const int* p : src) a.src[i++] = p;
    const int seq = ++h->rbSeq;
    k_readback<<<1, 64, 0, s>>>(a, h->rbHost, seq);
    *seqOut = seq;
    return hip_check(h, hipGetLastError(), "read-back kernel");
}

// Waits until the post of sequence `seq` or a later one has landed: the
// words then hold that post's values or a newer post's (the caller of a
// lagged read posts the same sources every time).
int read_back_wait(mas_context* h, hipStream_t s, int seq, int* out, int n) {
    auto landed = [&] { return __atomic_load_n(h->rbHost, __ATOMIC_ACQUIRE) - seq >= 0; };
    const auto t0 = std::chrono::steady_clock::now();
    while (!landed()) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
            int rc = hip_check(h, hipStreamSynchronize(s), "read-back sync");
            if (rc) return rc;
            if (!landed()) return fail(h, MAS_ERR_HIP, "read-back lost");
            break;
        }
    }
    for (int k = 0; k < n; ++k) out[k] = __atomic_load_n(h->rbHost + 1 + k, __ATOMIC_RELAXED);
    return MAS_OK;
}

int read_back(mas_context* h, hipStream_t s, std::initializer_list<const int*> src, int* out) {
    int seq = 0, rc = read_back_post(h, s, src, &seq);
    return rc ? rc : read_back_wait(h, s, seq, out, (int)src.size());
}

int pending_giveup(mas_context* h) {
    if (!h->c1Host) return MAS_OK;
    const int epoch = __atomic_exchange_n(h->c1Host, 0, __ATOMIC_ACQ_REL);
    if (epoch == 0) return MAS_OK;
    return fail(h, MAS_ERR_HIP, "apply #" + std::to_string((unsigned)epoch) + " (k_coarse1): a bounded hand-off wait "
                "gave up, so that apply's coarse part of z is incomplete (mas_stats.wait_timeouts counts the waits)");
}

static void release(Buffer& b) {
    if (b.p) hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

}  // namespace mas

using namespace mas;

#define MAS_TRY(x)                 \
    do {                           \
        int _rc = (x);             \
        if (_rc != MAS_OK) return _rc; \
    } while (0)

extern "C" {

int mas_version(void) { return MAS_ABI_VERSION; }

int mas_create(mas_handle* out, const mas_config* cfg) {
    if (!out) return MAS_ERR_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return MAS_ERR_NO_DEVICE;
    mas_context* h = new (std::nothrow) mas_context();
    if (!h) return MAS_ERR_NOMEM;
    if (cfg) h->cfg = *cfg;
    else h->cfg.device = -1;
    if (h->cfg.max_levels < 0 || h->cfg.resort_period < 0) {
        delete h;
        return MAS_ERR_ARG;
    }
    if (h->cfg.device >= 0) {
        if (h->cfg.device >= ndev || hipSetDevice(h->cfg.device) != hipSuccess) {
            delete h;
            return MAS_ERR_ARG;
        }
        h->device = h->cfg.device;
    } else {
        hipGetDevice(&h->device);
    }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess) {
        delete h;
        return MAS_ERR_HIP;
    }
    for (auto& e : h->ev) hipEventCreate(&e);
    {
        void* p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocCoherent) != hipSuccess) {
            mas_destroy(h);
            return MAS_ERR_HIP;
        }
        h->c1Host = static_cast<int*>(p);
        std::memset(p, 0, 64);
    }
    if (const char* v = std::getenv("MAS_FINE_VARIANT")) h->fineVariant = std::atoi(v);
    if (const char* v = std::getenv("MAS_INV_RESIDENT")) h->invResident = std::atoi(v) != 0;
    if (const char* v = std::getenv("MAS_RESIDENT_SPLIT")) h->residentSplit = std::atoi(v);
    if (const char* v = std::getenv("MAS_COARSE_OCC")) h->coarseOcc = std::atoi(v);
    if (const char* v = std::getenv("MAS_COARSE_NARROW")) h->coarseNarrow = std::atoi(v);
    if (const char* v = std::getenv("MAS_COARSE_WIDE")) h->coarseWide = std::atoi(v);
    if (const char* v = std::getenv("MAS_SORT")) h->sortImpl = std::atoi(v);
    if (h->cfg.reference_formation) h->factorVariant = 4;
    h->groupedR3 = !h->cfg.reference_restriction;
    if (const char* v = std::getenv("MAS_REF_RESTRICT")) h->groupedR3 = !std::atoi(v);
    if (const char* v = std::getenv("MAS_FACTOR_VARIANT")) h->factorVariant = std::atoi(v);
    if (const char* v = std::getenv("MAS_PCG_FUSE_P")) h->pcgFuseP = std::atoi(v) != 0;
    if (const char* v = std::getenv("MAS_PCG_SYM")) h->pcgSym = std::atoi(v) != 0;
    if (const char* v = std::getenv("MAS_RZ_WPB")) {
        const int w = std::atoi(v);
        h->rzWpb = (w == 4 || w == 8) ? w : 2;
    }
    if (const char* v = std::getenv("MAS_COARSE_MODE")) h->coarseMode = std::atoi(v);
    if (const char* v = std::getenv("MAS_C1_POLL_DELAY")) h->c1PollDelay = std::atoi(v);
    if (const char* v = std::getenv("MAS_C1_CHUNK")) h->c1Chunk = std::atoi(v);
    if (const char* v = std::getenv("MAS_C1_POLL_LIMIT")) h->c1PollLimit = std::atoi(v);
    if (const char* v = std::getenv("MAS_PREP_CU_RESERVE")) h->prepCuReserve = std::atoi(v);
    if (const char* v = std::getenv("MAS_FUSED_CHUNKS")) h->fusedChunks = std::atoi(v);
    if (const char* v = std::getenv("MAS_FUSED_AFTER_LEVELS")) h->fusedAfterLevels = std::atoi(v);
    if (const char* v = std::getenv("MAS_EARLY_THREAD")) h->earlyThread = std::atoi(v);
    if (const char* v = std::getenv("MAS_EARLY_OD")) h->earlyOd = std::atoi(v);
    if (const char* v = std::getenv("MAS_FOLD_SIDE")) h->foldSide = std::atoi(v);
    if (const char* v = std::getenv("MAS_HIER_CACHE")) h->hierCache = std::atoi(v);
    h->hostRegister = h->cfg.host_register;
    if (const char* v = std::getenv("MAS_HOST_REGISTER")) h->hostRegister = std::atoi(v);
    if (const char* v = std::getenv("MAS_SHARD_MODE")) h->shardMode = std::atoi(v);
    // MAS_PREP_SERIAL=1 (A/B) queues the early path on the caller's stream: from
    // one host thread, so the launch order on that stream is fixed
    if (const char* v = std::getenv("MAS_PREP_SERIAL"))
        if (std::atoi(v)) h->earlyThread = 0;
    int rc = upload_slot_table(h);
    if (rc == MAS_OK && (rc = ensure(h, h->devStatus, 16 * sizeof(int))) == MAS_OK)
        rc = hip_check(h, hipMemset(h->devStatus.p, 0, 16 * sizeof(int)), "device status words");
    if (rc != MAS_OK) {
        mas_destroy(h);
        return rc;
    }
    *out = h;
    return MAS_OK;
}

int mas_destroy(mas_handle h) {
    if (!h) return MAS_ERR_ARG;
    h->prepWorker.reset();  // idle between Prepares: joined before anything it used goes
    hipSetDevice(h->device);
    if (h->stream) hipStreamSynchronize(h->stream);
    // drain every stream this handle enqueued on -- including an allgather of
    // mas_shard_apply_rccl still writing shardGathered -- before the
    // communicator and the buffers go
    if (h->commStream) hipStreamSynchronize(h->commStream);
    if (h->evShardDone) hipEventSynchronize(h->evShardDone);
    if (h->prepStream) {
        hipStreamSynchronize(h->prepStream);
        hipStreamDestroy(h->prepStream);
    }
    if (h->evPrepFork) hipEventDestroy(h->evPrepFork);
    if (h->evPrepJoin) hipEventDestroy(h->evPrepJoin);
    if (h->evAdd0) hipEventDestroy(h->evAdd0);
    if (h->foldStream) {
        hipStreamSynchronize(h->foldStream);
        hipStreamDestroy(h->foldStream);
    }
    if (h->evFoldFork) hipEventDestroy(h->evFoldFork);
    if (h->evFoldJoin) hipEventDestroy(h->evFoldJoin);
    if (h->evDiag1) hipEventDestroy(h->evDiag1);
    if (h->evPreJoin) hipEventDestroy(h->evPreJoin);
    for (auto& e : h->evFine)
        if (e) hipEventDestroy(e);
    release_comm(h);  // drained above; the communicator goes before the buffers it wrote
    for (auto& q : h->pins)
        if (q.registered) hipHostUnregister(const_cast<void*>(q.p));
    (void)hipGetLastError();
    h->for_each_buffer([](Buffer& b) { release(b); });
    for (auto& e : h->ev)
        if (e) hipEventDestroy(e);
    for (auto& e : h->prof) hipEventDestroy(e);
    if (h->commStream) {
        hipStreamSynchronize(h->commStream);
        hipStreamDestroy(h->commStream);
    }
    if (h->evRestrict) hipEventDestroy(h->evRestrict);
    if (h->evGathered) hipEventDestroy(h->evGathered);
    if (h->evShardDone) hipEventDestroy(h->evShardDone);
    if (h->stream) hipStreamDestroy(h->stream);
    if (h->rbHost) hipHostFree(h->rbHost);
    if (h->c1Host) hipHostFree(h->c1Host);
    delete h;
    return MAS_OK;
}

const char* mas_last_error(mas_handle h) { return h ? h->err.c_str() : "null handle"; }

int mas_allocate(mas_handle h, int nV, int nE, int nF, const float* pos4, const int* nbr_starts, const int* nbr_idx,
                 const int* edges4, const int* faces4) {
    if (!h) return MAS_ERR_ARG;
    if (nV <= 0 || nE < 0 || nF < 0 || !pos4 || !nbr_starts || !nbr_idx)
        return fail(h, MAS_ERR_ARG, "mas_allocate: bad arguments");
    if (h->allocated && nV != h->nV)
        return fail(h, MAS_ERR_STATE, "mas_allocate: numVerts must stay fixed after the first call");
    hipSetDevice(h->device);
    if (h->fromBlob) {  // a restored handle starts over as a fresh one
        h->fromBlob = false;
        h->allocated = false;
        h->prepared = false;
        h->allocCalls = 0;
    }
    h->nE = nE;
    h->nF = nF;
    h->nV = nV;
    return run_allocate(h, pos4, nbr_starts, nbr_idx, edges4, faces4);
}

// Page-lock the caller's host array of slot `slot` (mas_context::pins) so the
// copies of the host-pointer entry points run at the pinned rate instead of
// through the runtime's pageable staging.  An array is registered the second
// time it comes back in the same slot (same pointer and size): a caller that
// passes a fresh temporary every call (a Python binding's output array) never
// pays a registration per call.  Memory that is pinned already (hipHostMalloc,
// a torch pinned tensor) or cannot be registered is used as it is:
// registration only changes the copy rate, never the result, and no error of
// these calls is left behind for the caller's next HIP check.
static void pin_host(mas_context* h, int slot, const void* p, size_t bytes) {
    if (!h->hostRegister || !p || !bytes) return;
    auto& q = h->pins[slot];
    if (q.p != p || q.bytes != bytes) {
        if (q.registered) {
            hipHostUnregister(const_cast<void*>(q.p));
            (void)hipGetLastError();  // the caller may have freed it already
        }
        q.p = p;
        q.bytes = bytes;
        q.registered = false;
        q.seen = 1;
        return;
    }
    if (q.registered || q.seen++ != 1) return;  // registered, or found unregistrable
    // page-aligned arrays only, registered to the end of their last page (the
    // caller's allocation covers it, mas_config.host_register): registering a
    // page shared with another allocation would pin, and let the runtime
    // treat as pinned, memory this handle knows nothing about
    if (reinterpret_cast<uintptr_t>(p) & 4095) return;
    for (const auto& o : h->pins)  // one registration per array (z and r may be one buffer)
        if (&o != &q && o.registered && o.p == p) return;
    hipPointerAttribute_t attr{};
    const bool pinned = hipPointerGetAttributes(&attr, p) == hipSuccess && attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();
    if (pinned) return;
    q.registered = hipHostRegister(const_cast<void*>(p), (bytes + 4095) & ~size_t(4095), hipHostRegisterDefault) ==
                   hipSuccess;
    (void)hipGetLastError();  // a refused registration leaves the copy pageable, not an error
}

static int prepare_common(mas_handle h, const float* d_diag9, const float* d_off9, const int* d_ranges, const void* ef,
                          const void* ee, const void* vf, const unsigned* efC, const unsigned* eeC,
                          const unsigned* vfC, hipStream_t s) {
    if (!h->allocated || h->fromBlob) return fail(h, MAS_ERR_STATE, "prepare before allocate");
    return run_prepare(h, d_diag9, d_off9, d_ranges, ef, ee, vf, efC, eeC, vfC, s);
}

int mas_prepare(mas_handle h, const float* diag9, const float* off9, const int* ranges, const void* ef, const void* ee,
                const void* vf, const unsigned* efC, const unsigned* eeC, const unsigned* vfC) {
    if (!h) return MAS_ERR_ARG;
    if (!diag9 || !off9 || !ranges) return fail(h, MAS_ERR_ARG, "mas_prepare: null Hessian pointer");
    if (!h->allocated || h->fromBlob) return fail(h, MAS_ERR_STATE, "prepare before allocate");
    hipSetDevice(h->device);
    const size_t nV = h->nV, nnz = h->nnz;
    MAS_TRY(ensure(h, h->diagStage, nV * 36));
    MAS_TRY(ensure(h, h->offStage, nnz * 36));
    MAS_TRY(ensure(h, h->rangeStage, (nV + 1) * 4));
    pin_host(h, 0, diag9, nV * 36);
    pin_host(h, 1, off9, nnz * 36);
    pin_host(h, 2, ranges, (nV + 1) * 4);
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->diagStage.p, diag9, nV * 36, hipMemcpyHostToDevice, h->stream), "H2D diag"));
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->offStage.p, off9, nnz * 36, hipMemcpyHostToDevice, h->stream), "H2D off"));
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->rangeStage.p, ranges, (nV + 1) * 4, hipMemcpyHostToDevice, h->stream),
                      "H2D ranges"));
    MAS_TRY(prepare_common(h, P<float>(h->diagStage), P<float>(h->offStage), P<int>(h->rangeStage), ef, ee, vf, efC,
                           eeC, vfC, h->stream));
    return hip_check(h, hipStreamSynchronize(h->stream), "prepare sync");
}

int mas_prepare_device(mas_handle h, const float* d_diag9, const float* d_off9, const int* d_ranges, const void* ef,
                       const void* ee, const void* vf, const unsigned* efC, const unsigned* eeC, const unsigned* vfC,
                       void* stream) {
    if (!h) return MAS_ERR_ARG;
    if (!d_diag9 || !d_off9 || !d_ranges) return fail(h, MAS_ERR_ARG, "mas_prepare_device: null Hessian pointer");
    hipSetDevice(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    return prepare_common(h, d_diag9, d_off9, d_ranges, ef, ee, vf, efC, eeC, vfC, s);
}

int mas_apply_device(mas_handle h, float* d_z4, const float* d_r4, void* stream) {
    if (!h) return MAS_ERR_ARG;
    if (!d_z4 || !d_r4) return fail(h, MAS_ERR_ARG, "mas_apply_device: null vector");
    if ((reinterpret_cast<uintptr_t>(d_z4) | reinterpret_cast<uintptr_t>(d_r4)) & 15)
        return fail(h, MAS_ERR_ARG, "mas_apply_device: vectors must be 16-byte aligned");
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    // an earlier apply (device or host) whose coarse hand-off gave up is
    // reported here, before this one is queued: its z was incomplete
    MAS_TRY(pending_giveup(h));
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    return run_apply(h, reinterpret_cast<float4*>(d_z4), reinterpret_cast<const float4*>(d_r4), s);
}

int mas_pcg_solve_device(mas_handle h, const float* d_diag9, const float* d_off9, const int* d_ranges, float* d_x4,
                         const float* d_b4, int max_iters, float tol, int precondition, mas_pcg_result* out,
                         void* stream) {
    if (!h) return MAS_ERR_ARG;
    if (!d_diag9 || !d_off9 || !d_ranges || !d_x4 || !d_b4)
        return fail(h, MAS_ERR_ARG, "mas_pcg_solve_device: null pointer");
    if ((reinterpret_cast<uintptr_t>(d_x4) | reinterpret_cast<uintptr_t>(d_b4)) & 15)
        return fail(h, MAS_ERR_ARG, "mas_pcg_solve_device: vectors must be 16-byte aligned");
    if (max_iters < 0 || !(tol >= 0.0f)) return fail(h, MAS_ERR_ARG, "mas_pcg_solve_device: bad max_iters / tol");
    if (precondition && !h->prepared) return fail(h, MAS_ERR_STATE, "preconditioned solve before prepare");
    if (!h->allocated || h->fromBlob) return fail(h, MAS_ERR_STATE, "solve before allocate (needs the neighbour ids)");
    hipSetDevice(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    return run_pcg(h, d_diag9, d_off9, d_ranges, reinterpret_cast<float4*>(d_x4),
                   reinterpret_cast<const float4*>(d_b4), max_iters, tol, precondition, out, s);
}

int mas_pcg_solve(mas_handle h, const float* diag9, const float* off9, const int* ranges, float* x4, const float* b4,
                  int max_iters, float tol, int precondition, mas_pcg_result* out) {
    if (!h) return MAS_ERR_ARG;
    if (!diag9 || !off9 || !ranges || !x4 || !b4) return fail(h, MAS_ERR_ARG, "mas_pcg_solve: null pointer");
    if (!h->allocated || h->fromBlob) return fail(h, MAS_ERR_STATE, "solve before allocate (needs the neighbour ids)");
    hipSetDevice(h->device);
    const size_t nV = h->nV, nnz = h->nnz, vb = nV * 16;
    MAS_TRY(ensure(h, h->diagStage, nV * 36));
    MAS_TRY(ensure(h, h->offStage, nnz * 36));
    MAS_TRY(ensure(h, h->rangeStage, (nV + 1) * 4));
    MAS_TRY(ensure(h, h->pcgStage, 2 * vb));
    pin_host(h, 0, diag9, nV * 36);
    pin_host(h, 1, off9, nnz * 36);
    pin_host(h, 2, ranges, (nV + 1) * 4);
    pin_host(h, 5, x4, vb);
    pin_host(h, 6, b4, vb);
    float* dx = P<float>(h->pcgStage);
    float* db = dx + 4 * nV;
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->diagStage.p, diag9, nV * 36, hipMemcpyHostToDevice, h->stream), "H2D diag"));
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->offStage.p, off9, nnz * 36, hipMemcpyHostToDevice, h->stream), "H2D off"));
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->rangeStage.p, ranges, (nV + 1) * 4, hipMemcpyHostToDevice, h->stream),
                      "H2D ranges"));
    MAS_TRY(hip_check(h, hipMemcpyAsync(dx, x4, vb, hipMemcpyHostToDevice, h->stream), "H2D x"));
    MAS_TRY(hip_check(h, hipMemcpyAsync(db, b4, vb, hipMemcpyHostToDevice, h->stream), "H2D b"));
    MAS_TRY(mas_pcg_solve_device(h, P<float>(h->diagStage), P<float>(h->offStage), P<int>(h->rangeStage), dx, db,
                                 max_iters, tol, precondition, out, h->stream));
    MAS_TRY(hip_check(h, hipMemcpyAsync(x4, dx, vb, hipMemcpyDeviceToHost, h->stream), "D2H x"));
    return hip_check(h, hipStreamSynchronize(h->stream), "solve sync");
}

int mas_apply(mas_handle h, float* z4, const float* r4) {
    if (!h) return MAS_ERR_ARG;
    if (!z4 || !r4) return fail(h, MAS_ERR_ARG, "mas_apply: null vector");
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "apply before prepare");
    MAS_TRY(pending_giveup(h));  // an earlier device apply's incomplete z, first
    hipSetDevice(h->device);
    const size_t bytes = (size_t)h->nV * 16;
    MAS_TRY(ensure(h, h->rStage, bytes));
    MAS_TRY(ensure(h, h->zStage, bytes));
    pin_host(h, 3, r4, bytes);
    pin_host(h, 4, z4, bytes);
    MAS_TRY(hip_check(h, hipMemcpyAsync(h->rStage.p, r4, bytes, hipMemcpyHostToDevice, h->stream), "H2D r"));
    MAS_TRY(run_apply(h, P<float4>(h->zStage), P<float4>(h->rStage), h->stream));
    MAS_TRY(hip_check(h, hipMemcpyAsync(z4, h->zStage.p, bytes, hipMemcpyDeviceToHost, h->stream), "D2H z"));
    MAS_TRY(hip_check(h, hipStreamSynchronize(h->stream), "apply sync"));
    return pending_giveup(h);  // a synchronous apply reports its own incomplete z
}

int mas_set_profiling(mas_handle h, int enable) {
    if (!h) return MAS_ERR_ARG;
    hipSetDevice(h->device);
    if (enable && h->prof.empty()) {
        h->prof.resize(4 * kProfRing);
        for (auto& e : h->prof)
            if (hipEventCreate(&e) != hipSuccess) return fail(h, MAS_ERR_HIP, "hipEventCreate");
    }
    if (h->stream) hipStreamSynchronize(h->stream);
    h->profiling = enable != 0;
    h->profRecorded = 0;
    h->stats.profiled_applies = 0;
    h->stats.apply_ms_avg = h->stats.pre_fine_ms_avg = h->stats.fine_ms_avg = h->stats.post_fine_ms_avg = 0.0;
    return MAS_OK;
}

int mas_profile_fine(mas_handle h, float* d_z4, const float* d_r4, int n, void* stream, double* ms_per_launch) {
    if (!h) return MAS_ERR_ARG;
    if (!d_z4 || !d_r4 || !ms_per_launch || n <= 0) return fail(h, MAS_ERR_ARG, "mas_profile_fine: bad arguments");
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "profile before prepare");
    if ((reinterpret_cast<uintptr_t>(d_z4) | reinterpret_cast<uintptr_t>(d_r4)) & 15)
        return fail(h, MAS_ERR_ARG, "mas_profile_fine: vectors must be 16-byte aligned");
    if (h->fineBlk0 != 0 || h->fineBlk1 != h->nFineBlk)
        return fail(h, MAS_ERR_STATE, "mas_profile_fine: the handle was prepared for one shard");
    hipSetDevice(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    ScopedEvents ev;
    if (!ev.ok()) return fail(h, MAS_ERR_HIP, "hipEventCreate");
    MAS_TRY(hip_check(h, hipEventRecord(ev.e[0], s), "record"));
    for (int i = 0; i < n; ++i)
        launch_fine(h, 0, h->nFineBlk, reinterpret_cast<const float4*>(d_r4), reinterpret_cast<float4*>(d_z4), s);
    MAS_TRY(hip_check(h, hipGetLastError(), "fine kernel"));
    MAS_TRY(hip_check(h, hipEventRecord(ev.e[1], s), "record"));
    MAS_TRY(hip_check(h, hipEventSynchronize(ev.e[1]), "profile sync"));
    float ms = 0.f;
    MAS_TRY(hip_check(h, hipEventElapsedTime(&ms, ev.e[0], ev.e[1]), "elapsed"));
    *ms_per_launch = (double)ms / n;
    return MAS_OK;
}

int mas_profile_coarse(mas_handle h, const float* d_r4, int n, void* stream, double* ms_per_launch) {
    if (!h) return MAS_ERR_ARG;
    if (!d_r4 || !ms_per_launch || n <= 0) return fail(h, MAS_ERR_ARG, "mas_profile_coarse: bad arguments");
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "profile before prepare");
    if (h->fineBlk0 != 0 || h->fineBlk1 != h->nFineBlk)
        return fail(h, MAS_ERR_STATE, "mas_profile_coarse: the handle was prepared for one shard");
    if (h->L < 2) return fail(h, MAS_ERR_STATE, "mas_profile_coarse: no coarse level");
    MAS_TRY(pending_giveup(h));
    hipSetDevice(h->device);
    hipStream_t s = stream ? (hipStream_t)stream : h->stream;
    ScopedEvents ev;
    if (!ev.ok()) return fail(h, MAS_ERR_HIP, "hipEventCreate");
    MAS_TRY(hip_check(h, hipEventRecord(ev.e[0], s), "record"));
    for (int i = 0; i < n; ++i) launch_coarse_apply(h, reinterpret_cast<const float4*>(d_r4), s);
    MAS_TRY(hip_check(h, hipGetLastError(), "coarse kernels"));
    MAS_TRY(hip_check(h, hipEventRecord(ev.e[1], s), "record"));
    MAS_TRY(hip_check(h, hipEventSynchronize(ev.e[1]), "profile sync"));
    float ms = 0.f;
    MAS_TRY(hip_check(h, hipEventElapsedTime(&ms, ev.e[0], ev.e[1]), "elapsed"));
    *ms_per_launch = (double)ms / n;
    return pending_giveup(h);
}

int mas_get_info(mas_handle h, mas_info* out) {
    if (!h || !out) return MAS_ERR_ARG;
    std::memset(out, 0, sizeof(*out));
    out->num_verts = h->nV;
    out->num_edges = h->nE;
    out->num_faces = h->nF;
    out->num_levels = h->L;
    out->natural_levels = h->natL;
    out->total_clusters = h->totalClusters;
    out->num_blocks = h->nBlk;
    out->num_fine_blocks = h->nFineBlk;
    out->max_neighbors = h->maxNbr;
    out->num_stencils = h->nStencil;
    std::memcpy(out->level_size, h->levelSize, sizeof(out->level_size));
    out->inv_bytes = (int64_t)h->nBlk * kBlockFloats * 4;
    h->for_each_buffer([&](Buffer& b) { out->device_bytes += (int64_t)b.bytes; });
    return MAS_OK;
}

int mas_get_stats(mas_handle h, mas_stats* out) {
    if (!h || !out) return MAS_ERR_ARG;
    const int n = std::min(h->profRecorded, kProfRing);
    if (n > 0) {
        hipSetDevice(h->device);
        double sa = 0, sr = 0, sc = 0, sf = 0;
        for (int i = 0; i < n; ++i) {
            hipEvent_t* e = &h->prof[4 * i];
            if (hipEventSynchronize(e[3]) != hipSuccess) return fail(h, MAS_ERR_HIP, "profiling event sync");
            float a = 0, r = 0, c = 0, f = 0;
            hipEventElapsedTime(&a, e[0], e[3]);
            hipEventElapsedTime(&r, e[0], e[1]);
            hipEventElapsedTime(&f, e[1], e[2]);
            hipEventElapsedTime(&c, e[2], e[3]);
            sa += a; sr += r; sc += c; sf += f;
        }
        h->stats.profiled_applies = n;
        h->stats.apply_ms_avg = sa / n;
        h->stats.pre_fine_ms_avg = sr / n;
        h->stats.fine_ms_avg = sf / n;
        h->stats.post_fine_ms_avg = sc / n;
    }
    h->stats.apply_mode = coarse_mode(h);
    if (h->c1Launched) {
        // the waits that gave up, counted on the device since mas_create, read
        // on the handle's own stream: no device-wide synchronisation (applies
        // still running on another stream may add to it later; each apply
        // that gives up is also reported by the next call, pending_giveup)
        hipSetDevice(h->device);
        int n = 0;
        if (hipMemcpyAsync(&n, P<int>(h->devStatus) + 2, 4, hipMemcpyDeviceToHost, h->stream) != hipSuccess ||
            hipStreamSynchronize(h->stream) != hipSuccess)
            return fail(h, MAS_ERR_HIP, "mas_get_stats: reading the wait counter");
        h->stats.wait_timeouts = n;
    }
    *out = h->stats;
    return MAS_OK;
}

int mas_get_maps(mas_handle h, uint64_t* morton, int* s2o, int* o2s, int* cst, int* going_next, int* coarse_tables,
                 unsigned* fine_mask) {
    if (!h) return MAS_ERR_ARG;
    if (!h->allocated) return fail(h, MAS_ERR_STATE, "maps before allocate");
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    const size_t nV = h->nV;
    auto cp = [&](void* dst, const Buffer& b, size_t bytes) -> int {
        if (!dst) return MAS_OK;
        if (!b.p || b.bytes < bytes) return fail(h, MAS_ERR_STATE, "map not computed yet");
        return hip_check(h, hipMemcpy(dst, b.p, bytes, hipMemcpyDeviceToHost), "D2H maps");
    };
    MAS_TRY(cp(morton, h->morton, nV * 8));
    MAS_TRY(cp(s2o, h->s2o, nV * 4));
    MAS_TRY(cp(o2s, h->o2s, nV * 4));
    if (cst || going_next || coarse_tables || fine_mask) {
        if (!h->prepared) return fail(h, MAS_ERR_STATE, "level maps before prepare");
        MAS_TRY(cp(cst, h->cst, (size_t)h->L * nV * 4));
        MAS_TRY(cp(going_next, h->goingNext, (size_t)h->totalClusters * 4));
        MAS_TRY(cp(coarse_tables, h->coarseTables, nV * 16));
        MAS_TRY(cp(fine_mask, h->fineMask, nV * 4));
    }
    return MAS_OK;
}

int mas_get_neighbors(mas_handle h, int* nbr_num, int* nbr) {
    if (!h) return MAS_ERR_ARG;
    if (!h->allocated || !h->nbr.p || h->fromBlob) return fail(h, MAS_ERR_STATE, "neighbors before allocate");
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    if (nbr_num) MAS_TRY(hip_check(h, hipMemcpy(nbr_num, h->nbrNum.p, (size_t)h->nV * 4, hipMemcpyDeviceToHost), "D2H"));
    if (nbr)
        MAS_TRY(hip_check(h, hipMemcpy(nbr, h->nbr.p, (size_t)h->maxNbr * h->nV * 4, hipMemcpyDeviceToHost), "D2H"));
    return MAS_OK;
}

// a coarse block of a Prepare with the coarse split exists only where the
// rank factored it (its pre / post ranges, coarse_split.hip), post blocks only
// after the exchange
static int coarse_block_ready(mas_handle h, int blk) {
    if (!h->splitPlanned || blk < h->nFineBlk) return MAS_OK;
    for (size_t i = 0; i + 1 < h->splitPre.size(); i += 2)
        if (blk >= h->splitPre[i] && blk < h->splitPre[i + 1]) return MAS_OK;
    for (size_t i = 0; i + 1 < h->splitPost.size(); i += 2)
        if (blk >= h->splitPost[i] && blk < h->splitPost[i + 1])
            return h->rowsPending ? fail(h, MAS_ERR_STATE, "coarse block of a sharded Prepare before the exchange "
                                                           "(mas_prepare_shard_complete)")
                                  : MAS_OK;
    return fail(h, MAS_ERR_STATE, "coarse block another rank of this sharded Prepare assembles");
}

int mas_get_block_matrix(mas_handle h, int blk, float* out96) {
    if (!h || !out96) return MAS_ERR_ARG;
    if (!h->prepared || h->fromBlob || !h->dense.p)
        return fail(h, MAS_ERR_STATE, "block matrix before prepare (a restored blob holds no assembly blocks)");
    if (blk < 0 || blk >= h->nBlk) return fail(h, MAS_ERR_ARG, "block index out of range");
    if (blk < h->nFineBlk && (blk < h->fineBlk0 || blk >= h->fineBlk1))
        return fail(h, MAS_ERR_STATE, "level-0 block outside the shard this handle was prepared for");
    MAS_TRY(coarse_block_ready(h, blk));
    if (blk < h->nFineBlk && !h->denseFine)
        return fail(h, MAS_ERR_STATE, "level-0 blocks are not stored by the fused assemble + factor "
                                      "(create the handle with mas_config.keep_blocks = 1)");
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    MAS_TRY(hip_check(h, hipMemcpy(out96, dense_base(h) + (size_t)blk * kDenseFloats, kDenseFloats * 4,
                                   hipMemcpyDeviceToHost), "D2H block"));
    // zero-diagonal -> identity rule (.cpp:1365-1368), as the factor kernel applies it
    for (int x = 0; x < 32; ++x) {
        if (out96[(3 * x) * 96 + 3 * x] != 0.0f) continue;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) out96[(3 * x + i) * 96 + 3 * x + j] = (i == j) ? 1.f : 0.f;
    }
    return MAS_OK;
}

int mas_get_block_inverse(mas_handle h, int blk, float* out96) {
    if (!h || !out96) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "block inverse before prepare");
    if (blk < 0 || blk >= h->nBlk) return fail(h, MAS_ERR_ARG, "block index out of range");
    if (blk < h->nFineBlk && (blk < h->fineBlk0 || blk >= h->fineBlk1))
        return fail(h, MAS_ERR_STATE, "level-0 block outside the shard this handle was prepared for");
    MAS_TRY(coarse_block_ready(h, blk));
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    return copy_block_inverse(h, blk, out96);
}

int mas_get_packed_inverses(mas_handle h, int blk0, int nblk, float* out) {
    if (!h || !out || nblk < 0) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "inverses before prepare");
    if (blk0 < 0 || blk0 + nblk > h->nBlk) return fail(h, MAS_ERR_ARG, "block range out of range");
    for (int b = blk0; b < blk0 + nblk; ++b) {
        if (b < h->nFineBlk && (b < h->fineBlk0 || b >= h->fineBlk1))
            return fail(h, MAS_ERR_STATE, "level-0 block outside the shard this handle was prepared for");
        MAS_TRY(coarse_block_ready(h, b));
    }
    hipSetDevice(h->device);
    hipStreamSynchronize(h->stream);
    return hip_check(h, hipMemcpy(out, P<float>(h->inv) + (size_t)blk0 * kBlockFloats,
                                  (size_t)nblk * kBlockFloats * 4, hipMemcpyDeviceToHost), "D2H inverses");
}

int mas_get_coarse_residual(mas_handle h, float* out4) {
    if (!h || !out4) return MAS_ERR_ARG;
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "coarse residual before prepare");
    const int nCoarse = h->totalClusters - h->levelSize[3];
    if (nCoarse <= 0) return MAS_OK;
    hipSetDevice(h->device);
    hipDeviceSynchronize();  // the apply may have run on any stream
    return hip_check(h, hipMemcpy(out4, h->Rc.p, (size_t)nCoarse * 16, hipMemcpyDeviceToHost), "D2H Rc");
}

int mas_set_prepare_shard(mas_handle h, int rank, int world) {
    if (!h) return MAS_ERR_ARG;
    if (world < 1 || rank < 0 || rank >= world) return fail(h, MAS_ERR_ARG, "mas_set_prepare_shard: bad rank/world");
    h->prepRank = rank;
    h->prepWorld = world;
    return MAS_OK;
}

}  // extern "C"

int mas_dev_sort_pairs(mas_handle h, const unsigned* d_keys_in, unsigned* d_keys_out, const int* d_vals_in,
                       int* d_vals_out, int n, int bits, int impl) {
    if (!h || n < 0 || (n > 0 && (!d_keys_in || !d_keys_out || !d_vals_in || !d_vals_out))) return MAS_ERR_ARG;
    hipSetDevice(h->device);
    const int keep = h->sortImpl;
    h->sortImpl = impl;
    const int rc = mas::sort_pairs_u32(h, d_keys_in, d_keys_out, d_vals_in, d_vals_out, n, bits, h->stream, "sort");
    h->sortImpl = keep;
    if (rc) return rc;
    return hip_check(h, hipStreamSynchronize(h->stream), "sort");
}

int mas_dev_exclusive_scan(mas_handle h, const int* d_in, int* d_out, int n, int impl) {
    if (!h || n < 0 || (n > 0 && (!d_in || !d_out))) return MAS_ERR_ARG;
    hipSetDevice(h->device);
    int rc;
    if (impl) {
        rc = mas::rs_exclusive_scan(h, d_in, d_out, n, h->stream, "scan");
    } else {
        size_t tmp = 0;
        hipcub::DeviceScan::ExclusiveSum(nullptr, tmp, d_in, d_out, n, h->stream);
        rc = ensure(h, h->cubTemp, tmp);
        if (!rc)
            rc = hip_check(h, hipcub::DeviceScan::ExclusiveSum(h->cubTemp.p, tmp, d_in, d_out, n, h->stream), "scan");
    }
    if (rc) return rc;
    return hip_check(h, hipStreamSynchronize(h->stream), "scan");
}
