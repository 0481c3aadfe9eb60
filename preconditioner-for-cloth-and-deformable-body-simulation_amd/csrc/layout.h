// layout.h -- the packed layout of one 32-node subdomain inverse (4656 fp32).
//
// The reference packs the symmetric 96x96 inverse as a diagonal plus 8-wide
// diagonal strips plus a scalar remainder (.cpp:1435-1495), shaped for AVX2.
// On CDNA4 one wave64 solves one block: lane L = 32 h + n owns node n, and the
// two halves h split the 3x3 node-pair blocks G(n, m) = Inv[3n..3n+2][3m..3m+2]
// by rotation distance s = (m - n) mod 32:
//
//   half 0, lane n: record f  0..62   G(n, n+1+k), k = 0..6   (f = 9k + 3a + b)
//                          f 63..65   s = 16: n < 16 row 0 of G(n, n+16),
//                                             n >= 16 row 1 of G(n-16, n)
//                          f 66..71   D(n) upper triangle (00 01 02 11 12 22)
//   half 1, lane n: record f  0..71   G(n, n+8+k), k = 0..7   (f = 9k + 3a + b)
//   tail (48 floats)                  row 2 of G(p, p+16), p = 0..15 (3p + b)
//
// Memory: float4 q (0..17) of lane L at float4 index q*64 + L, then the tail.
// 18*64*4 + 48 = 4656 floats = 18 624 B: exactly the reference's packed size;
// every wave-instruction of the apply kernel reads 1 KiB contiguous, and each
// lane finds every value it multiplies in its own registers.
#pragma once

namespace mas {

constexpr int kMainFloats = 18 * 64 * 4;  // 4608
constexpr int kRecord = 72;               // floats per lane

// (i, j), i <= j: the Inv entry stored at float offset o of a packed block.
__host__ __device__ inline void slot_ij(int o, int& i, int& j) {
    int r, c;
    if (o < kMainFloats) {
        const int F = o >> 2, comp = o & 3;
        const int q = F >> 6, L = F & 63, h = L >> 5, n = L & 31;
        const int f = 4 * q + comp;
        if (h == 1 || f < 63) {
            const int k = f / 9, e = f % 9;
            const int s = h ? 8 + k : 1 + k;
            const int m = (n + s) & 31;
            r = 3 * n + e / 3;
            c = 3 * m + e % 3;
        } else if (f < 66) {
            const int b = f - 63;
            if (n < 16) {
                r = 3 * n;
                c = 3 * (n + 16) + b;
            } else {
                r = 3 * (n - 16) + 1;
                c = 3 * n + b;
            }
        } else {
            const int d = f - 66;
            const int a = (d < 3) ? 0 : (d < 5 ? 1 : 2);
            const int b = (d < 3) ? d : (d < 5 ? d - 2 : 2);
            r = 3 * n + a;
            c = 3 * n + b;
        }
    } else {
        const int t = o - kMainFloats, p = t / 3, b = t % 3;
        r = 3 * p + 2;
        c = 3 * (p + 16) + b;
    }
    i = r < c ? r : c;
    j = r < c ? c : r;
}

// Inverse of slot_ij: the float offset of Inv entry (i, j) (either order).
__host__ __device__ inline int slot_of(int i, int j) {
    int ni = i / 3, nj = j / 3, a = i % 3, b = j % 3;
    auto at = [](int f, int h, int n) { return ((f >> 2) * 64 + 32 * h + n) * 4 + (f & 3); };
    if (ni == nj) {  // D(n) upper triangle, half 0, f = 66 + (00 01 02 11 12 22)
        if (a > b) { const int x = a; a = b; b = x; }
        const int d = a == 0 ? b : (a == 1 ? 2 + b : 5);
        return at(66 + d, 0, ni);
    }
    int s = (nj - ni) & 31;
    if (s > 16) {  // stored from the other node: G(m, n) = G(n, m)^T
        int x = ni; ni = nj; nj = x;
        x = a; a = b; b = x;
        s = 32 - s;
    }
    if (s == 16) {
        if (ni >= 16) {  // orient as G(p, p + 16), p < 16
            int x = ni; ni = nj; nj = x;
            x = a; a = b; b = x;
        }
        if (a == 0) return at(63 + b, 0, ni);
        if (a == 1) return at(63 + b, 0, ni + 16);
        return kMainFloats + 3 * ni + b;
    }
    const int e = 3 * a + b;
    if (s <= 7) return at(9 * (s - 1) + e, 0, ni);
    return at(9 * (s - 8) + e, 1, ni);
}

}  // namespace mas
