// rsort.hip -- the stable (u32 key, int) radix sort and the int exclusive scan
// of Prepare, without decoupled look-back.
//
// Why not rocprim: its onesweep sort and look-back scan make each workgroup
// wait on its predecessor's published prefix.  Beside the fused level-0 kernel
// (prepStream), whose gathers keep the memory system busy, those waits stalled
// for the fused kernel's whole duration -- a 95k-key onesweep pass took
// 2.76 ms instead of 20 us (profiles/round3/prepare, scripts/dev/sort_overlap.hip
// reproduces it with a memory-streaming kernel on another stream).  Here every
// workgroup only depends on the previous kernel of its own stream.
//
// Sort, per pass of `nb` <= 8 key bits (ceil(bits / 8) passes, equal widths):
//   k_rs_count      tiles of 4096 keys (256 threads x 16, striped): per-tile
//                   digit counts -> hist[digit][tile]
//   k_rs_digit_scan one workgroup per digit: exclusive scan along the tiles,
//                   the digit's total
//   k_rs_scatter    tile base = scan of the digit totals + hist[digit][tile];
//                   rank within the tile in (round, wave, lane) = input order:
//                   a wave's equal-digit lanes found by nb ballots, their
//                   counts per (round, wave) slot prefix-summed per digit
// Stable, so the output permutation is unique: equal to rocprim's bit for bit
// (tests/test_gpu_rsort.py).
//
// Scan: reduce (tile sums) -> one-workgroup scan of the sums -> down-sweep.
#include <hip/hip_runtime.h>

#include "mas_internal.h"

namespace mas {

namespace {

constexpr int kRsThreads = 256, kRsItems = 16, kRsTile = kRsThreads * kRsItems;
constexpr int kRsSlots = kRsItems * (kRsThreads / 64);  // (round, wave) slots per tile

// exclusive scan of one int per thread over the workgroup; *total = the sum
template <int THREADS>
__device__ __forceinline__ int block_scan_excl(int v, int* wsum, int* total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    int inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    int before = 0, all = 0;
#pragma unroll
    for (int k = 0; k < THREADS / 64; ++k) {
        const int s = wsum[k];
        before += k < w ? s : 0;
        all += s;
    }
    __syncthreads();  // wsum is reused by the caller's next scan
    *total = all;
    return before + inc - v;
}

// lanes of this wave whose digit equals d (valid lanes only)
__device__ __forceinline__ unsigned long long peer_mask(unsigned d, bool valid, int nb) {
    unsigned long long m = __ballot(valid);
    for (int b = 0; b < nb; ++b) {
        const bool bit = (d >> b) & 1u;
        const unsigned long long bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__global__ __launch_bounds__(kRsThreads) void k_rs_count(const unsigned* __restrict__ keys, int n, int shift, int nb,
                                                          int* __restrict__ hist, int nTiles) {
    __shared__ int cnt[256];
    const int t = threadIdx.x, lane = t & 63;
    const unsigned mask = (1u << nb) - 1u;
    const long long base = (long long)blockIdx.x * kRsTile;
    cnt[t] = 0;
    unsigned k[kRsItems];
#pragma unroll
    for (int r = 0; r < kRsItems; ++r) {
        const long long i = base + r * kRsThreads + t;
        k[r] = i < n ? keys[i] : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRsItems; ++r) {
        const bool valid = base + r * kRsThreads + t < n;
        const unsigned d = (k[r] >> shift) & mask;
        const unsigned long long m = peer_mask(d, valid, nb);
        if (valid && lane == __ffsll((long long)m) - 1) atomicAdd(&cnt[d], __popcll(m));
    }
    __syncthreads();
    if ((unsigned)t <= mask) hist[(size_t)t * nTiles + blockIdx.x] = cnt[t];
}

__global__ __launch_bounds__(kRsThreads) void k_rs_digit_scan(int* __restrict__ hist, int nTiles,
                                                               int* __restrict__ digitTot) {
    __shared__ int wsum[kRsThreads / 64];
    const int t = threadIdx.x;
    int* row = hist + (size_t)blockIdx.x * nTiles;
    const int per = (nTiles + kRsThreads - 1) / kRsThreads;
    const int j0 = t * per, j1 = min(j0 + per, nTiles);
    int sum = 0;
    for (int j = j0; j < j1; ++j) sum += row[j];
    int total = 0;
    int run = block_scan_excl<kRsThreads>(sum, wsum, &total);
    for (int j = j0; j < j1; ++j) {
        const int v = row[j];
        row[j] = run;
        run += v;
    }
    if (t == 0) digitTot[blockIdx.x] = total;
}

__global__ __launch_bounds__(kRsThreads) void k_rs_scatter(const unsigned* __restrict__ kin,
                                                            const int* __restrict__ vin, unsigned* __restrict__ kout,
                                                            int* __restrict__ vout, int n, int shift, int nb,
                                                            const int* __restrict__ hist,
                                                            const int* __restrict__ digitTot, int nTiles) {
    __shared__ __attribute__((aligned(16))) unsigned short cnt[kRsSlots][256];
    __shared__ int base[256];
    __shared__ int wsum[kRsThreads / 64];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int bins = 1 << nb;
    const unsigned mask = (unsigned)bins - 1u;
    const long long tile0 = (long long)blockIdx.x * kRsTile;
    {
        uint4* c4 = reinterpret_cast<uint4*>(&cnt[0][0]);
        constexpr int n4 = kRsSlots * 256 * 2 / 16;
#pragma unroll
        for (int q = 0; q < n4 / kRsThreads; ++q) c4[q * kRsThreads + t] = make_uint4(0, 0, 0, 0);
    }
    unsigned k[kRsItems];
    int v[kRsItems];
#pragma unroll
    for (int r = 0; r < kRsItems; ++r) {
        const long long i = tile0 + r * kRsThreads + t;
        k[r] = i < n ? kin[i] : 0u;
        v[r] = i < n ? vin[i] : 0;
    }
    {
        const int tot = t < bins ? digitTot[t] : 0;
        int all = 0;
        const int excl = block_scan_excl<kRsThreads>(tot, wsum, &all);  // its barriers also order the zeroing
        if (t < bins) base[t] = excl + hist[(size_t)t * nTiles + blockIdx.x];
    }
    unsigned rankDigit[kRsItems];  // rank within the wave << 8 | digit
    const unsigned long long lt = (1ull << lane) - 1ull;
#pragma unroll
    for (int r = 0; r < kRsItems; ++r) {
        const bool valid = tile0 + r * kRsThreads + t < n;
        const unsigned d = (k[r] >> shift) & mask;
        const unsigned long long m = peer_mask(d, valid, nb);
        rankDigit[r] = ((unsigned)__popcll(m & lt) << 8) | d;
        if (valid && lane == __ffsll((long long)m) - 1) cnt[r * 4 + w][d] = (unsigned short)__popcll(m);
    }
    __syncthreads();
    if (t < bins) {
        // in batches of 16 slots (loads in flight together; ~50 VGPRs, so the
        // kernel fits beside the fused level-0 waves)
        int run = 0;
#pragma unroll
        for (int q0 = 0; q0 < kRsSlots; q0 += 16) {
            int c[16];
#pragma unroll
            for (int q = 0; q < 16; ++q) c[q] = cnt[q0 + q][t];
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                cnt[q0 + q][t] = (unsigned short)run;
                run += c[q];
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kRsItems; ++r) {
        if (tile0 + r * kRsThreads + t < n) {
            const unsigned d = rankDigit[r] & 0xffu;
            const int pos = base[d] + cnt[r * 4 + w][d] + (int)(rankDigit[r] >> 8);
            kout[pos] = k[r];
            vout[pos] = v[r];
        }
    }
}

constexpr int kScanThreads = 256, kScanItems = 16, kScanTile = kScanThreads * kScanItems;

template <bool VEC>
__device__ __forceinline__ void scan_load(const int* __restrict__ in, long long i0, int n, int (&x)[kScanItems]) {
    if (VEC && i0 + kScanItems <= n) {
        const int4* p = reinterpret_cast<const int4*>(in + i0);
#pragma unroll
        for (int q = 0; q < kScanItems / 4; ++q) {
            const int4 a = p[q];
            x[4 * q] = a.x; x[4 * q + 1] = a.y; x[4 * q + 2] = a.z; x[4 * q + 3] = a.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < kScanItems; ++q) x[q] = i0 + q < n ? in[i0 + q] : 0;
    }
}

template <bool VEC>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const int* __restrict__ in, int n,
                                                               int* __restrict__ part) {
    __shared__ int wsum[kScanThreads / 64];
    int x[kScanItems];
    scan_load<VEC>(in, (long long)blockIdx.x * kScanTile + threadIdx.x * kScanItems, n, x);
    int s = 0;
#pragma unroll
    for (int q = 0; q < kScanItems; ++q) s += x[q];
    int total = 0;
    block_scan_excl<kScanThreads>(s, wsum, &total);
    if (threadIdx.x == 0) part[blockIdx.x] = total;
}

// one workgroup: exclusive scan of the tile sums in place
__global__ __launch_bounds__(1024) void k_scan_top(int* __restrict__ part, int nb) {
    __shared__ int wsum[16];
    const int t = threadIdx.x;
    const int per = (nb + 1023) / 1024;
    const int j0 = t * per, j1 = min(j0 + per, nb);
    int sum = 0;
    for (int j = j0; j < j1; ++j) sum += part[j];
    int total = 0;
    int run = block_scan_excl<1024>(sum, wsum, &total);
    for (int j = j0; j < j1; ++j) {
        const int v = part[j];
        part[j] = run;
        run += v;
    }
}

template <bool VEC>
__global__ __launch_bounds__(kScanThreads) void k_scan_down(const int* in, int* out, int n,
                                                             const int* __restrict__ part) {
    __shared__ int wsum[kScanThreads / 64];
    const long long i0 = (long long)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    int x[kScanItems];
    scan_load<VEC>(in, i0, n, x);
    int s = 0;
#pragma unroll
    for (int q = 0; q < kScanItems; ++q) s += x[q];
    int total = 0;
    int run = block_scan_excl<kScanThreads>(s, wsum, &total) + (part ? part[blockIdx.x] : 0);
    int y[kScanItems];
#pragma unroll
    for (int q = 0; q < kScanItems; ++q) {
        y[q] = run;
        run += x[q];
    }
    if (VEC && i0 + kScanItems <= n) {
        int4* p = reinterpret_cast<int4*>(out + i0);
#pragma unroll
        for (int q = 0; q < kScanItems / 4; ++q) p[q] = make_int4(y[4 * q], y[4 * q + 1], y[4 * q + 2], y[4 * q + 3]);
    } else {
#pragma unroll
        for (int q = 0; q < kScanItems; ++q)
            if (i0 + q < n) out[i0 + q] = y[q];
    }
}

}  // namespace

int rs_sort_pairs(mas_context* h, const unsigned* kin, unsigned* kout, const int* vin, int* vout, int n, int bits,
                  hipStream_t s, const char* what, bool side) {
    Buffer& sKeys = side ? h->rsKeysP : h->rsKeys;
    Buffer& sVals = side ? h->rsValsP : h->rsVals;
    Buffer& sHist = side ? h->rsHistP : h->rsHist;
    if (n <= 0) return MAS_OK;
    if (bits <= 0) {  // no key bits: the input order
        int rc = hip_check(h, hipMemcpyAsync(kout, kin, (size_t)n * 4, hipMemcpyDeviceToDevice, s), what);
        return rc ? rc : hip_check(h, hipMemcpyAsync(vout, vin, (size_t)n * 4, hipMemcpyDeviceToDevice, s), what);
    }
    if (bits > 32) return fail(h, MAS_ERR_ARG, "radix sort: more than 32 key bits");
    const int passes = (bits + 7) / 8, per = (bits + passes - 1) / passes;
    const int nTiles = (int)(((long long)n + kRsTile - 1) / kRsTile);
    int rc;
    if ((passes > 1 && ((rc = ensure(h, sKeys, (size_t)n * 4)) || (rc = ensure(h, sVals, (size_t)n * 4)))) ||
        (rc = ensure(h, sHist, ((size_t)nTiles * 256 + 256) * 4)))
        return rc;
    int* hist = P<int>(sHist);
    int* digitTot = hist + (size_t)nTiles * 256;
    const unsigned* ki = kin;
    const int* vi = vin;
    for (int p = 0; p < passes; ++p) {
        const int shift = p * per, nb = std::min(per, bits - shift);
        // the last pass writes kout; earlier ones alternate back from it
        const bool toOut = (passes - 1 - p) % 2 == 0;
        unsigned* ko = toOut ? kout : P<unsigned>(sKeys);
        int* vo = toOut ? vout : P<int>(sVals);
        k_rs_count<<<nTiles, kRsThreads, 0, s>>>(ki, n, shift, nb, hist, nTiles);
        k_rs_digit_scan<<<1 << nb, kRsThreads, 0, s>>>(hist, nTiles, digitTot);
        k_rs_scatter<<<nTiles, kRsThreads, 0, s>>>(ki, vi, ko, vo, n, shift, nb, hist, digitTot, nTiles);
        ki = ko;
        vi = vo;
    }
    return hip_check(h, hipGetLastError(), what);
}

int rs_exclusive_scan(mas_context* h, const int* in, int* out, int n, hipStream_t s, const char* what, bool side) {
    if (n <= 0) return MAS_OK;
    const int nb = (int)(((long long)n + kScanTile - 1) / kScanTile);
    const bool vec = ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
    int* part = nullptr;
    if (nb > 1) {
        Buffer& sPart = side ? h->rsPartP : h->rsPart;
        int rc = ensure(h, sPart, (size_t)nb * 4);
        if (rc) return rc;
        part = P<int>(sPart);
        if (vec) k_scan_reduce<true><<<nb, kScanThreads, 0, s>>>(in, n, part);
        else k_scan_reduce<false><<<nb, kScanThreads, 0, s>>>(in, n, part);
        k_scan_top<<<1, 1024, 0, s>>>(part, nb);
    }
    if (vec) k_scan_down<true><<<nb, kScanThreads, 0, s>>>(in, out, n, part);
    else k_scan_down<false><<<nb, kScanThreads, 0, s>>>(in, out, n, part);
    return hip_check(h, hipGetLastError(), what);
}

}  // namespace mas
