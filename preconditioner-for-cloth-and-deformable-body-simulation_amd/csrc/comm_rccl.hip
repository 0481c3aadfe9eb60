// comm_rccl.hip -- RCCL (xGMI) allgather for the one-call sharded apply
// (mas_shard_apply_rccl, include/mas_capi.h; SURVEY §8(e): "the small
// coarse-level residuals exchanged via RCCL allgather over xGMI").
//
// RCCL is bound at run time: dlopen("librccl.so.1") returns the copy already
// in the process when there is one (torch-ROCm loads its own under the same
// soname), so a Python process and a plain C++ simulator both work and the
// library has no link-time RCCL dependency.  The communicator belongs to the
// handle (mas_rccl_init) and is destroyed with it.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <mutex>
#include <string>

#include "mas_internal.h"

namespace mas {

struct RcclApi {
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclAllGather) allGather = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
    std::string why;
    bool ok() const { return getUniqueId && commInitRank && commDestroy && allGather && errorString; }
};

static const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* so = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) so = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!so) {
            const char* e = dlerror();
            api.why = std::string("librccl.so.1 not loadable: ") + (e ? e : "?");
            return;
        }
        api.getUniqueId = reinterpret_cast<decltype(api.getUniqueId)>(dlsym(so, "ncclGetUniqueId"));
        api.commInitRank = reinterpret_cast<decltype(api.commInitRank)>(dlsym(so, "ncclCommInitRank"));
        api.commDestroy = reinterpret_cast<decltype(api.commDestroy)>(dlsym(so, "ncclCommDestroy"));
        api.allGather = reinterpret_cast<decltype(api.allGather)>(dlsym(so, "ncclAllGather"));
        api.errorString = reinterpret_cast<decltype(api.errorString)>(dlsym(so, "ncclGetErrorString"));
        if (!api.ok()) api.why = "librccl.so.1 lacks an entry point";
    });
    return api;
}

void release_comm(mas_context* h) {
    if (h->rcclComm && rccl().ok()) rccl().commDestroy(static_cast<ncclComm_t>(h->rcclComm));
    h->rcclComm = nullptr;
    h->rcclRank = -1;
    h->rcclWorld = 0;
}

// mas_allgather_fn over the handle's communicator: bytes are float4 segments
static int rccl_allgather(const void* send, void* recv, size_t bytes, void* stream, void* user) {
    mas_context* h = static_cast<mas_context*>(user);
    const ncclResult_t r = rccl().allGather(send, recv, bytes / sizeof(float), ncclFloat,
                                            static_cast<ncclComm_t>(h->rcclComm), static_cast<hipStream_t>(stream));
    if (r != ncclSuccess) {
        h->err = std::string("ncclAllGather: ") + rccl().errorString(r);
        return (int)r;
    }
    return 0;
}

int comm_allgather(mas_context* h, const void* send, void* recv, size_t bytes, hipStream_t s) {
    if (!h->rcclComm || !rccl().ok()) return fail(h, MAS_ERR_STATE, "no RCCL communicator (mas_rccl_init)");
    if (rccl_allgather(send, recv, bytes, s, h)) return fail(h, MAS_ERR_COMM, h->err);
    return MAS_OK;
}

}  // namespace mas

using namespace mas;

extern "C" {

int mas_rccl_unique_id(void* id128) {
    if (!id128) return MAS_ERR_ARG;
    const RcclApi& api = rccl();
    if (!api.ok()) return MAS_ERR_COMM;
    ncclUniqueId id;
    if (api.getUniqueId(&id) != ncclSuccess) return MAS_ERR_COMM;
    static_assert(sizeof(id) == 128, "ncclUniqueId is 128 bytes");
    __builtin_memcpy(id128, &id, sizeof(id));
    return MAS_OK;
}

int mas_rccl_init(mas_handle h, const void* id128, int rank, int world) {
    if (!h) return MAS_ERR_ARG;
    if (!id128 || world <= 0 || rank < 0 || rank >= world) return fail(h, MAS_ERR_ARG, "mas_rccl_init: bad arguments");
    const RcclApi& api = rccl();
    if (!api.ok()) return fail(h, MAS_ERR_COMM, api.why);
    hipSetDevice(h->device);
    release_comm(h);
    ncclUniqueId id;
    __builtin_memcpy(&id, id128, sizeof(id));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = api.commInitRank(&comm, world, id, rank);
    if (r != ncclSuccess) return fail(h, MAS_ERR_COMM, std::string("ncclCommInitRank: ") + api.errorString(r));
    h->rcclComm = comm;
    h->rcclRank = rank;
    h->rcclWorld = world;
    return MAS_OK;
}

int mas_shard_apply_rccl(mas_handle h, float* d_z4, const float* d_r4, void* stream) {
    if (!h) return MAS_ERR_ARG;
    if (!h->rcclComm) return fail(h, MAS_ERR_STATE, "mas_shard_apply_rccl before mas_rccl_init");
    return mas_shard_apply_device(h, h->rcclRank, h->rcclWorld, rccl_allgather, h, d_z4, d_r4, stream);
}

}  // extern "C"
