// ref_headers.cpp -- TEST INFRASTRUCTURE (never linked into the product).
//
// A harness over the reference's OWN, UNMODIFIED headers, compiled from where
// they lie under /root/reference by oracle/build_ref.sh into
// oracle/_ref/libref_headers.so.  Nothing is copied, patched or shimmed: the
// only prelude is <math.h>, which the reference's headers use without
// including (SeMath.h:87-99 calls logf/fabs/... ).
//
// What it pins (tests/golden/make_ref_fixtures.py turns it into fixtures):
//   * SeMorton64::Encode (SeMorton.h:75-86) and ExpandBits (:94-101), through
//     the reference's own Math::Clamp / Min / Max (SeMath.h:100-103,
//     SePreDefine.h:37-38) -- the B-8 NaN-to-hi clamp included;
//   * FillSortingData's normalisation t = (p - Lower) / Extent()
//     (SeSchwarzPreconditioner.cpp:219-235) with SeAabb::operator+= / Extent
//     (SeAabb.h:76-94) over SeVector3<float> (SeVector.h:215-...), the scalar
//     form of the SeVec3fSimd lanes (SSE min/max return the second operand on
//     NaN exactly like SE_MIN/SE_MAX's ternaries; SSE add/sub/div are the
//     IEEE scalar operations per lane);
//   * memory layouts of SeMatrix3f (SeMatrix.h:650-682), Int4 (SeVector.h:395),
//     Float2/Float3/Float4 and SeCsr<int> (SeCsr.h:35-173) with Size / IdxPtr.
//
//   * the contact Hessian terms of PrepareCollisionHessian /
//     AdditionalSchwarzHessian2 (SeSchwarzPreconditioner.cpp:1190,1208-1223):
//     the same expressions on the reference's own types -- Float3 d * stiff
//     (SeVector.h:250), OuterProduct (SeMatrix.h:352-363), Math::Square
//     (SeMath.h:98), SeMatrix3f * scalar and scalar * SeMatrix3f
//     (SeMatrix.h:741,977) -- written by element accessor (i, j).
//
// What it cannot pin: SeVec3fSimd and the contact records (SeVectorSimd.h and
// SeCollisionElements.h need a source patch of SeVectorSimd.h:101-102 to
// compile) and the .cpp's other floating-point phases (same patch + MSVC
// <intrin.h>); see DESIGN.md section 2.
#include <math.h>

#include "SeAabb.h"
#include "SeCsr.h"
#include "SeMath.h"
#include "SeMatrix.h"
#include "SeMorton.h"
#include "SeVector.h"

#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

namespace {

struct CsrProbe : SE::SeCsr<int> {
    CsrProbe(const std::vector<int>& s, const std::vector<int>& i) : SE::SeCsr<int>(s, i, {}) {}
    long long off(const void* member) const {
        return (long long)((const char*)member - (const char*)static_cast<const SE::SeCsr<int>*>(this));
    }
    long long off_starts() const { return off(&m_starts); }
    long long off_idxs() const { return off(&m_idxs); }
    long long off_values() const { return off(&m_values); }
};

struct LayoutRow {
    const char* name;
    long long value;
};

std::vector<LayoutRow> layout_rows() {
    std::vector<LayoutRow> r;
    r.push_back({"SeMatrix3f.sizeof", (long long)sizeof(SE::SeMatrix3f)});
    r.push_back({"SeMatrix3f.alignof", (long long)alignof(SE::SeMatrix3f)});
    r.push_back({"Int4.sizeof", (long long)sizeof(SE::Int4)});
    r.push_back({"Int4.alignof", (long long)alignof(SE::Int4)});
    r.push_back({"Int2.sizeof", (long long)sizeof(SE::Int2)});
    r.push_back({"Int2.alignof", (long long)alignof(SE::Int2)});
    r.push_back({"Float2.sizeof", (long long)sizeof(SE::Float2)});
    r.push_back({"Float2.alignof", (long long)alignof(SE::Float2)});
    r.push_back({"Float3.sizeof", (long long)sizeof(SE::Float3)});
    r.push_back({"Float3.alignof", (long long)alignof(SE::Float3)});
    r.push_back({"Float4.sizeof", (long long)sizeof(SE::Float4)});
    r.push_back({"Float4.alignof", (long long)alignof(SE::Float4)});
    r.push_back({"SeMorton64.sizeof", (long long)sizeof(SE::SeMorton64)});
    r.push_back({"SeMorton64.alignof", (long long)alignof(SE::SeMorton64)});
    r.push_back({"SeCsr<int>.sizeof", (long long)sizeof(SE::SeCsr<int>)});
    r.push_back({"SeCsr<int>.alignof", (long long)alignof(SE::SeCsr<int>)});
    CsrProbe p({0, 2, 3}, {1, 2, 0});
    r.push_back({"SeCsr<int>.offsetof.m_starts", p.off_starts()});
    r.push_back({"SeCsr<int>.offsetof.m_idxs", p.off_idxs()});
    r.push_back({"SeCsr<int>.offsetof.m_values", p.off_values()});
    // SeMatrix3f element (i, j): its float index inside the 36-byte object.
    SE::SeMatrix3f m(0.0f);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m(i, j) = (float)(10 * i + j);
    float raw[9];
    std::memcpy(raw, &m, sizeof(raw));
    static char names[9][32];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            int where = -1;
            for (int k = 0; k < 9; ++k)
                if (raw[k] == (float)(10 * i + j)) where = k;
            std::snprintf(names[3 * i + j], sizeof(names[0]), "SeMatrix3f.index(%d,%d)", i, j);
            r.push_back({names[3 * i + j], where});
        }
    return r;
}

}  // namespace

extern "C" {

// SeMorton64::Encode(x, y, z) (SeMorton.h:75-86), full 21-bit precision.
uint64_t refh_morton_encode(float x, float y, float z) {
    SE::SeMorton64 m;
    m.Encode(x, y, z);
    return (uint64_t)(SE::SeMorton64::value_type)m;
}

// Math::Clamp / Min / Max (SeMath.h:100-103) on float.
float refh_clamp(float a, float lo, float hi) { return SE::Math::Clamp(a, lo, hi); }
float refh_min(float a, float b) { return SE::Math::Min(a, b); }
float refh_max(float a, float b) { return SE::Math::Max(a, b); }

// ComputeAABB + FillSortingData (SeSchwarzPreconditioner.cpp:201-235) over
// pos4 = n x {x, y, z, w} (w ignored, as in SeVec3fSimd's xyz lanes).
// box6 <- {Lower.xyz, Upper.xyz}; codes[v] <- the Morton code of vertex v.
void refh_morton_points(const float* pos4, int n, uint64_t* codes, float* box6) {
    SE::SeAabb<SE::Float3> box;
    for (int v = 0; v < n; ++v) box += SE::Float3(pos4[4 * v], pos4[4 * v + 1], pos4[4 * v + 2]);
    const SE::Float3 ext = box.Extent();
    for (int v = 0; v < n; ++v) {
        SE::Float3 t = (SE::Float3(pos4[4 * v], pos4[4 * v + 1], pos4[4 * v + 2]) - box.Lower) / ext;
        SE::SeMorton64 m;
        m.Encode(t.x, t.y, t.z);
        codes[v] = (uint64_t)(SE::SeMorton64::value_type)m;
    }
    if (box6) {
        box6[0] = box.Lower.x, box6[1] = box.Lower.y, box6[2] = box.Lower.z;
        box6[3] = box.Upper.x, box6[4] = box.Upper.y, box6[5] = box.Upper.z;
    }
}

// Layout table: row i -> (name, value); returns 0 past the end.
int refh_layout(int i, const char** name, long long* value) {
    static const std::vector<LayoutRow> rows = layout_rows();
    if (i < 0 || i >= (int)rows.size()) return 0;
    *name = rows[i].name;
    *value = rows[i].value;
    return 1;
}

// SeCsr<int>(starts, idxs): Rows(), Size(), and per row Size(id) and
// IdxPtr(id) - IdxPtr(0) (SeCsr.h:114-142).
int refh_csr_probe(const int* starts, int rows, const int* idx, int* sizes, long long* idx_off, int* total) {
    std::vector<int> s(starts, starts + rows + 1), ix(idx, idx + starts[rows]);
    SE::SeCsr<int> c(s, ix, {});
    for (int r = 0; r < rows; ++r) {
        sizes[r] = c.Size(r);
        idx_off[r] = (long long)(c.IdxPtr(r) - c.IdxPtr(0));
    }
    *total = c.Size();
    return c.Rows();
}

// The contact terms of one stencil, as .cpp:1208-1223 and :1190 write them
// (the weights come from the stencil; here any five): out[234] column-major
// 3x3 each -- [0, 9) hessian = OuterProduct(d, d * s.stiff); [9 + 9 it]
// hessian * Math::Square(w[it]); [54 + 9 p] w[a] * w[b] * hessian and
// [144 + 9 p] that * 2.0f, pairs p over a < b < 5 in (a, b) order.
void refh_contact_terms(const float* dir3, float stiff, const float* w, float* out) {
    auto put = [&](const SE::SeMatrix3f& m, float* dst) {
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) dst[j * 3 + i] = m(i, j);
    };
    SE::Float3 d(dir3[0], dir3[1], dir3[2]);
    SE::SeMatrix3f hessian = SE::OuterProduct(d, d * stiff);
    put(hessian, out);
    for (int it = 0; it < 5; ++it) put(hessian * SE::Math::Square(w[it]), out + 9 + 9 * it);
    for (int a = 0, p = 0; a < 5; ++a)
        for (int b = a + 1; b < 5; ++b, ++p) {
            SE::SeMatrix3f t = w[a] * w[b] * hessian;
            put(t, out + 54 + 9 * p);
            put(t * 2.0f, out + 144 + 9 * p);
        }
}

}  // extern "C"
