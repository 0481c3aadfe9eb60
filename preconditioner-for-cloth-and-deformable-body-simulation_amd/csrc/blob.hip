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
    if (h->fineBlk0 != 0 || h->fineBlk1 != h->nFineBlk)
        return fail(h, MAS_ERR_STATE, "blob of a shard-prepared handle (not every block is factored)");
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

// Index-map checks of a blob whose checksum matched (FNV-1a detects
// corruption, not tampering): every id the apply kernels gather through must
// be in range, so a crafted blob cannot steer a GPU gather out of bounds.
static bool blob_maps_valid(const MasBlobHeader& hd, const unsigned char* in, const MasBlobSection* sec[]) {
    const int nV = hd.nV, L = hd.L, tc = hd.totalClusters;
    const int* ls = hd.levelSize;
    // level table: entry l >= 1 = (n_l, begin_l), begin_1 = ceil32(nV),
    // begin_{l+1} = begin_l + ceil32(n_l), total = begin_L (entry 0 is unused)
    if (ls[3] != (nV + 31) / 32 * 32) return false;
    for (int l = 1; l < L; ++l) {
        const long long n = ls[2 * l], b = ls[2 * l + 1];
        if (n <= 0 || n > (l == 1 ? nV : ls[2 * (l - 1)]) || b + (n + 31) / 32 * 32 != ls[2 * (l + 1) + 1])
            return false;
    }
    if (ls[2 * L + 1] != tc) return false;
    auto count = [&](int l) { return l == 0 ? nV : ls[2 * l]; };
    auto arr = [&](int i) { return reinterpret_cast<const int*>(in + sec[i]->offset); };
    std::vector<int> seen((size_t)nV, 0);
    const int* s2o = arr(kSecS2o);
    const int* o2s = arr(kSecO2s);
    for (int v = 0; v < nV; ++v) {
        if (s2o[v] < 0 || s2o[v] >= nV || seen[s2o[v]]++ || o2s[s2o[v]] != v) return false;
    }
    // goingNext of the real nodes below the top level: into the next level's
    // real nodes (top-level and padding entries are never followed)
    const int* gn = arr(kSecGoingNext);
    for (int l = 0; l + 1 < L; ++l) {
        const int b = l == 0 ? 0 : ls[2 * l + 1], nb = ls[2 * (l + 1) + 1];
        for (int i = b; i < b + count(l); ++i)
            if (gn[i] < nb || gn[i] >= nb + count(l + 1)) return false;
    }
    const int* cst = arr(kSecCst);
    for (int l = 0; l < L; ++l)
        for (int v = 0; v < nV; ++v) {
            const int c = cst[(size_t)l * nV + v];
            if (c < 0 || (l + 1 < L && c >= count(l + 1))) return false;
        }
    const int* ct = arr(kSecCoarseTables);  // ancestors of levels 1 .. L-1 (Int4, .cpp:1119-1147)
    for (int v = 0; v < nV; ++v)
        for (int l = 1; l < L && l <= 4; ++l)
            if (ct[4 * (size_t)v + l - 1] < ls[2 * l + 1] || ct[4 * (size_t)v + l - 1] >= ls[2 * l + 1] + count(l))
                return false;
    // per-vertex apply map {s2o, a1, a2, a3}: ancestors of the prolonged levels
    const int4* vm = reinterpret_cast<const int4*>(in + sec[kSecVmap]->offset);
    const int np = L < 4 ? L : 4;
    for (int v = 0; v < nV; ++v) {
        const int a[4] = {vm[v].x, vm[v].y, vm[v].z, vm[v].w};
        if (a[0] != s2o[v]) return false;
        for (int l = 1; l < np; ++l)
            if (a[l] < ls[2 * l + 1] || a[l] >= ls[2 * l + 1] + count(l)) return false;
    }
    // coarse members (child bank, component mask): inside the child level
    const int begin1 = ls[3];
    const int2* mb = reinterpret_cast<const int2*>(in + sec[kSecMembers]->offset);
    for (int l = 1; l < L; ++l) {
        const int nChild = count(l - 1);
        for (int p = 0; p < (count(l) + 31) / 32 * 32; ++p) {
            const int2 m = mb[ls[2 * l + 1] + p - begin1];
            if (m.x < 0 || (m.y != 0 && 32LL * m.x + 32 - __builtin_clz((unsigned)m.y) > nChild)) return false;
            if (p >= count(l) && m.y != 0) return false;  // padding nodes have no children
        }
    }
    // level-1 segment starts per level-0 bank: 0 .. n1, nondecreasing
    const int* f = arr(kSecL1First);
    const int n1 = L > 1 ? count(1) : 0;
    for (int b = 0; b <= hd.nFineBlk; ++b)
        if (f[b] < 0 || f[b] > n1 || (b > 0 && f[b] < f[b - 1])) return false;
    return f[hd.nFineBlk] == n1;
}

// Header, checksum, section table and index maps; no device work, nothing
// of a handle is touched.  On success sec[id] points at each section entry.
static int blob_parse(const unsigned char* in, size_t size, MasBlobHeader& hd, const MasBlobSection* sec[],
                      std::vector<MasBlobSection>& table, std::string& why) {
    auto bad = [&](const char* m) { why = m; return MAS_ERR_ARG; };
    if (!in || size < sizeof(hd)) return bad("blob: too short");
    std::memcpy(&hd, in, sizeof(hd));
    if (std::memcmp(hd.magic, kBlobMagic, 8) != 0) return bad("blob: bad magic");
    if (hd.version != kBlobVersion) return bad("blob: unsupported version");
    if (hd.headerBytes < sizeof(hd) || hd.headerBytes > size || hd.nSections <= 0 || hd.nSections > 64 ||
        hd.headerBytes + hd.payloadBytes != size)
        return bad("blob: inconsistent sizes");
    if (fnv1a(in + hd.headerBytes, size - hd.headerBytes) != hd.checksum) return bad("blob: checksum mismatch");
    if (hd.nV <= 0 || hd.L < 1 || hd.L > kMaxLevels || hd.nBlk <= 0 || hd.nFineBlk != (hd.nV + 31) / 32 ||
        hd.totalClusters != 32 * hd.nBlk || hd.levelSize[3] < 0 || hd.levelSize[3] > hd.totalClusters)
        return bad("blob: inconsistent header");
    table.resize(hd.nSections);
    if (hd.headerBytes + table.size() * sizeof(MasBlobSection) > size) return bad("blob: table");
    std::memcpy(table.data(), in + hd.headerBytes, table.size() * sizeof(MasBlobSection));
    // the sizes every section must have, from the header alone (a scratch context)
    mas_context probe;
    probe.nV = hd.nV; probe.L = hd.L; probe.totalClusters = hd.totalClusters;
    probe.nBlk = hd.nBlk; probe.nFineBlk = hd.nFineBlk;
    std::memcpy(probe.levelSize, hd.levelSize, sizeof(probe.levelSize));
    for (auto& d : sections(&probe)) {
        const MasBlobSection* t = nullptr;
        for (auto& e : table)
            if (e.id == d.id) t = &e;
        if (!t || t->bytes != d.bytes || t->offset % 16 || t->offset > size || t->bytes > size - t->offset)
            return bad("blob: section");
        sec[d.id] = t;
    }
    if (!blob_maps_valid(hd, in, sec)) return bad("blob: index maps out of range");
    return MAS_OK;
}

int blob_load(mas_context* h, const void* src, size_t size) {
    const unsigned char* in = static_cast<const unsigned char*>(src);
    MasBlobHeader hd;
    const MasBlobSection* sec[kSecInv + 1] = {};
    std::vector<MasBlobSection> table;
    std::string why;
    if (blob_parse(in, size, hd, sec, table, why) != MAS_OK) return fail(h, MAS_ERR_ARG, why);
    // commit: adopt the sizes, then upload every section
    h->prepared = false;
    h->allocated = false;
    // the restored maps are a hierarchy of their own: nothing cached applies
    h->meshHierValid = h->liveIsMesh = false;
    h->hierId = ++h->hierCounter;
    h->recHierId = ~0ull;
    h->nV = hd.nV; h->nE = hd.nE; h->nF = hd.nF; h->L = hd.L; h->natL = hd.natL;
    h->totalClusters = hd.totalClusters; h->nBlk = hd.nBlk; h->nFineBlk = hd.nFineBlk;
    h->fineBlk0 = 0; h->fineBlk1 = hd.nFineBlk;  // a blob holds every block's inverse
    h->maxNbr = hd.maxNbr; h->nStencil = hd.nStencil;
    std::memcpy(h->levelSize, hd.levelSize, sizeof(h->levelSize));
    const auto secs = sections(h);
    int rc;
    for (auto& d : secs) {
        const MasBlobSection* t = sec[d.id];
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
    h->tabHierId = h->hierId;
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

int mas_blob_validate(const void* src, size_t size) {
    MasBlobHeader hd;
    const MasBlobSection* sec[kSecInv + 1] = {};
    std::vector<MasBlobSection> table;
    std::string why;
    return blob_parse(static_cast<const unsigned char*>(src), size, hd, sec, table, why);
}

int mas_load_blob(mas_handle h, const void* src, size_t size) {
    if (!h) return MAS_ERR_ARG;
    hipSetDevice(h->device);
    return blob_load(h, src, size);
}

}  // extern "C"
