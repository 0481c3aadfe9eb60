// blob.hip -- versioned fixture / wire format of a prepared handle
// ("an on-disk fixture and wire format (versioned .mas blob:
// maps plus packed factors) ... used for cross-box golden comparison and for
// warm-starting Prepare").
//
// Layout (little endian, every section 16-byte aligned):
//   header   MasBlobHeader: magic "MASBLOB\0", version, sizes, level table,
//            section count, FNV-1a 64 of every byte after the header
//   table    nSections x MasBlobSection {id, bytes, offset}
//   payload  the sections, in table order
// Sections are the Allocate/Prepare results the apply and the map
// introspection read: Morton codes, both permutations, CoarseSpaceTables,
// goingNext, coarseTables, fine connect masks, the per-vertex apply map, the
// coarse member table, the level-1 segment starts (sharding) and the packed
// inverses.  The dense assembly blocks and the neighbour table are Prepare
// intermediates and are not stored: a restored handle applies, shards and
// reports its maps and inverses, and needs mas_allocate before a new Prepare.
#include <cstring>
#include <vector>

#include "mas_internal.h"

namespace mas {

constexpr char kBlobMagic[8] = {'M', 'A', 'S', 'B', 'L', 'O', 'B', 0};
constexpr uint32_t kBlobVersion = 1;

struct MasBlobHeader {
    char magic[8];
    uint32_t version, headerBytes;
    int32_t nV, nE, nF, L, natL, totalClusters, nBlk, nFineBlk, maxNbr, nStencil;
    int32_t levelSize[2 * 9];
    int32_t nSections, reserved;
    uint64_t payloadBytes, checksum;
};

struct MasBlobSection {
    uint32_t id, pad;
    uint64_t bytes, offset;  // offset from the blob start
};

enum BlobSectionId : uint32_t {
    kSecMorton = 1, kSecS2o, kSecO2s, kSecCst, kSecGoingNext, kSecCoarseTables, kSecFineMask,
    kSecVmap, kSecMembers, kSecL1First, kSecInv
};

static uint64_t fnv1a(const unsigned char* p, size_t n, uint64_t h = 1469598103934665603ull) {
    for (size_t i = 0; i < n; ++i) {
        h ^= p[i];
        h *= 1099511628211ull;
    }
    return h;
}

static size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

struct SecDesc {
    uint32_t id;
    Buffer* buf;            // device buffer (nullptr: host vector l1First)
    size_t bytes;
};

static std::vector<SecDesc> sections(mas_context* h) {
    const size_t nV = h->nV;
    const int nCoarse = h->totalClusters - h->levelSize[3];
    std::vector<SecDesc> s = {
        {kSecMorton, &h->morton, nV * 8},
        {kSecS2o, &h->s2o, nV * 4},
        {kSecO2s, &h->o2s, nV * 4},
        {kSecCst, &h->cst, (size_t)h->L * nV * 4},
        {kSecGoingNext, &h->goingNext, (size_t)h->totalClusters * 4},
        {kSecCoarseTables, &h->coarseTables, nV * 16},
        {kSecFineMask, &h->fineMask, nV * 4},
        {kSecVmap, &h->vmap, nV * 16},
        {kSecMembers, &h->members, (size_t)(nCoarse > 0 ? nCoarse : 0) * 8},
        {kSecL1First, nullptr, (size_t)(h->nFineBlk + 1) * 4},
        {kSecInv, &h->inv, (size_t)h->nBlk * kBlockFloats * 4},
    };
    return s;
}

int blob_size(mas_context* h, size_t* out) {
    if (!h->prepared) return fail(h, MAS_ERR_STATE, "blob of an unprepared handle");
    auto secs = sections(h);
    size_t n = align16(sizeof(MasBlobHeader)) + align16(secs.size() * sizeof(MasBlobSection));
    for (auto& d : secs) n += align16(d.bytes);
    *out = n;
    return MAS_OK;
}

int blob_save(mas_context* h, void* dst, size_t cap, size_t* written) {
    size_t need = 0;
    int rc = blob_size(h, &need);
    if (rc) return rc;
    if (!dst || cap < need) return fail(h, MAS_ERR_CAPACITY, "blob buffer too small (see mas_blob_size)");
    if ((rc = hip_check(h, hipStreamSynchronize(h->stream), "blob sync"))) return rc;
    unsigned char* out = static_cast<unsigned char*>(dst);
    std::memset(out, 0, need);
    auto secs = sections(h);
    MasBlobHeader hd{};
    std::memcpy(hd.magic, kBlobMagic, 8);
    hd.version = kBlobVersion;
    hd.headerBytes = (uint32_t)align16(sizeof(MasBlobHeader));
    hd.nV = h->nV; hd.nE = h->nE; hd.nF = h->nF; hd.L = h->L; hd.natL = h->natL;
    hd.totalClusters = h->totalClusters; hd.nBlk = h->nBlk; hd.nFineBlk = h->nFineBlk;
    hd.maxNbr = h->maxNbr; hd.nStencil = h->nStencil;
    std::memcpy(hd.levelSize, h->levelSize, sizeof(hd.levelSize));
    hd.nSections = (int32_t)secs.size();
    const size_t tableAt = hd.headerBytes;
    size_t at = tableAt + align16(secs.size() * sizeof(MasBlobSection));
    const size_t payloadAt = tableAt;
    std::vector<MasBlobSection> table(secs.size());
    for (size_t i = 0; i < secs.size(); ++i) {
        table[i] = MasBlobSection{secs[i].id, 0, secs[i].bytes, at};
        if (secs[i].bytes) {
            if (secs[i].buf) {
                if (!secs[i].buf->p || secs[i].buf->bytes < secs[i].bytes)
                    return fail(h, MAS_ERR_STATE, "blob: a section is missing on the device");
                if ((rc = hip_check(h, hipMemcpy(out + at, secs[i].buf->p, secs[i].bytes, hipMemcpyDeviceToHost),
                                    "D2H blob section")))
                    return rc;
            } else {
                std::memcpy(out + at, h->l1First.data(), secs[i].bytes);
            }
        }
        at += align16(secs[i].bytes);
    }
    std::memcpy(out + tableAt, table.data(), table.size() * sizeof(MasBlobSection));
    hd.payloadBytes = need - payloadAt;
    hd.checksum = fnv1a(out + payloadAt, need - payloadAt);
    std::memcpy(out, &hd, sizeof(hd));
    if (written) *written = need;
    return MAS_OK;
}

int blob_load(mas_context* h, const void* src, size_t size) {
    const unsigned char* in = static_cast<const unsigned char*>(src);
    MasBlobHeader hd;
    if (!src || size < sizeof(hd)) return fail(h, MAS_ERR_ARG, "blob: too short");
    std::memcpy(&hd, in, sizeof(hd));
    if (std::memcmp(hd.magic, kBlobMagic, 8) != 0) return fail(h, MAS_ERR_ARG, "blob: bad magic");
    if (hd.version != kBlobVersion) return fail(h, MAS_ERR_ARG, "blob: unsupported version");
    if (hd.headerBytes < sizeof(hd) || hd.headerBytes > size || hd.nSections <= 0 || hd.nSections > 64 ||
        hd.headerBytes + hd.payloadBytes != size)
        return fail(h, MAS_ERR_ARG, "blob: inconsistent sizes");
    if (fnv1a(in + hd.headerBytes, size - hd.headerBytes) != hd.checksum)
        return fail(h, MAS_ERR_ARG, "blob: checksum mismatch");
    if (hd.nV <= 0 || hd.L < 1 || hd.L > kMaxLevels || hd.nBlk <= 0 || hd.nFineBlk != (hd.nV + 31) / 32 ||
        hd.totalClusters != 32 * hd.nBlk)
        return fail(h, MAS_ERR_ARG, "blob: inconsistent header");
    std::vector<MasBlobSection> table(hd.nSections);
    if (hd.headerBytes + table.size() * sizeof(MasBlobSection) > size) return fail(h, MAS_ERR_ARG, "blob: table");
    std::memcpy(table.data(), in + hd.headerBytes, table.size() * sizeof(MasBlobSection));
    // adopt the sizes, then every section must have exactly the size this handle expects
    h->prepared = false;
    h->allocated = false;
    h->nV = hd.nV; h->nE = hd.nE; h->nF = hd.nF; h->L = hd.L; h->natL = hd.natL;
    h->totalClusters = hd.totalClusters; h->nBlk = hd.nBlk; h->nFineBlk = hd.nFineBlk;
    h->maxNbr = hd.maxNbr; h->nStencil = hd.nStencil;
    std::memcpy(h->levelSize, hd.levelSize, sizeof(h->levelSize));
    auto secs = sections(h);
    int rc;
    for (auto& d : secs) {
        const MasBlobSection* t = nullptr;
        for (auto& e : table)
            if (e.id == d.id) t = &e;
        if (!t || t->bytes != d.bytes || t->offset + t->bytes > size) return fail(h, MAS_ERR_ARG, "blob: section");
        if (d.buf) {
            if ((rc = ensure(h, *d.buf, d.bytes ? d.bytes : 16))) return rc;
            if (d.bytes &&
                (rc = hip_check(h, hipMemcpy(d.buf->p, in + t->offset, d.bytes, hipMemcpyHostToDevice), "H2D blob")))
                return rc;
        } else {
            h->l1First.assign(h->nFineBlk + 1, 0);
            std::memcpy(h->l1First.data(), in + t->offset, d.bytes);
        }
    }
    const int nCoarse = h->totalClusters - h->levelSize[3];
    if ((rc = ensure(h, h->Rc, (size_t)(nCoarse > 0 ? nCoarse : 1) * 16)) ||
        (rc = ensure(h, h->Zc, (size_t)(nCoarse > 0 ? nCoarse : 1) * 16)))
        return rc;
    if (nCoarse > 0 && (rc = hip_check(h, hipMemset(h->Rc.p, 0, (size_t)nCoarse * 16), "memset Rc"))) return rc;
    if ((rc = build_l1src(h, h->stream)) || (rc = hip_check(h, hipStreamSynchronize(h->stream), "blob sync")))
        return rc;
    h->shardWorld = 0;
    h->fromBlob = true;
    h->allocated = true;  // maps are valid
    h->prepared = true;
    return MAS_OK;
}

}  // namespace mas

using namespace mas;

extern "C" {

int mas_blob_size(mas_handle h, size_t* out_bytes) {
    if (!h || !out_bytes) return MAS_ERR_ARG;
    return blob_size(h, out_bytes);
}

int mas_save_blob(mas_handle h, void* dst, size_t capacity, size_t* written) {
    if (!h) return MAS_ERR_ARG;
    hipSetDevice(h->device);
    if (h->prepared && h->l1First.empty())  // computed lazily after Prepare (k_shard.hip)
        if (int rc = compute_l1_first(h, h->stream)) return rc;
    return blob_save(h, dst, capacity, written);
}

int mas_load_blob(mas_handle h, const void* src, size_t size) {
    if (!h) return MAS_ERR_ARG;
    hipSetDevice(h->device);
    return blob_load(h, src, size);
}

}  // extern "C"
