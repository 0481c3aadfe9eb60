// The facade's value types against the layouts the reference's OWN headers
// produce (tests/golden/ref_headers.json, made by
// tests/golden/make_ref_fixtures.py from SeMatrix.h / SeVector.h / SeCsr.h /
// SeMorton.h).  ref_layout_values.h is generated from that fixture by
// tests/test_ref_pinned.py; every REF_* macro is a value measured on the
// reference's types.  Compile-time asserts for sizes / alignments / offsets,
// a run-time check for SeMatrix3f's element order and SeCsr::Size / IdxPtr.
#include <cstddef>
#include <cstdio>
#include <cstring>
#include <vector>

#include "SeSchwarzPreconditioner.h"
#include "ref_layout_values.h"

using namespace SE;

static_assert(sizeof(SeMatrix3f) == REF_SeMatrix3f_sizeof && alignof(SeMatrix3f) == REF_SeMatrix3f_alignof,
              "SeMatrix3f");
static_assert(sizeof(Int4) == REF_Int4_sizeof && alignof(Int4) == REF_Int4_alignof, "Int4");
static_assert(sizeof(Float2) == REF_Float2_sizeof && alignof(Float2) == REF_Float2_alignof, "Float2");
static_assert(sizeof(Float3) == REF_Float3_sizeof && alignof(Float3) == REF_Float3_alignof, "Float3");
static_assert(sizeof(SeCsr<int>) == REF_SeCsr_int_sizeof && alignof(SeCsr<int>) == REF_SeCsr_int_alignof,
              "SeCsr<int>");
// The contact records embed Float2 / Float3 at the offsets the reference's
// field order gives; their own headers cannot be compiled unpatched, so the
// record offsets are derived from the pinned member types here.
static_assert(offsetof(EfSet, m_bary) == 12 && offsetof(EfSet, m_bary) % REF_Float3_alignof == 0, "EfSet bary");
static_assert(offsetof(VfSet, m_bary) == 16 && offsetof(VfSet, m_bary) % REF_Float2_alignof == 0, "VfSet bary");
static_assert(offsetof(EeSet, m_bary) == 16 && offsetof(EeSet, m_bary) % REF_Float2_alignof == 0, "EeSet bary");

struct CsrProbe : SeCsr<int> {
    CsrProbe(const std::vector<int>& s, const std::vector<int>& i) : SeCsr<int>(s, i, {}) {}
    long off(const void* m) const { return (long)((const char*)m - (const char*)static_cast<const SeCsr<int>*>(this)); }
    long off_starts() const { return off(&m_starts); }
    long off_idxs() const { return off(&m_idxs); }
    long off_values() const { return off(&m_values); }
};

int main() {
    int bad = 0;
    // SeMatrix3f element order
    SeMatrix3f m(0.f);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) m(i, j) = (float)(10 * i + j);
    float raw[9];
    std::memcpy(raw, &m, sizeof(raw));
    const int index[3][3] = REF_SeMatrix3f_index;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            if (raw[index[i][j]] != (float)(10 * i + j)) {
                std::printf("SeMatrix3f (%d,%d) not at %d\n", i, j, index[i][j]);
                bad = 1;
            }
    // SeCsr<int> member offsets and Size / IdxPtr on the fixture CSR
    const std::vector<int> starts = REF_CSR_STARTS, idx = REF_CSR_IDX;
    CsrProbe p(starts, idx);
    if (p.off_starts() != REF_SeCsr_int_off_starts || p.off_idxs() != REF_SeCsr_int_off_idxs ||
        p.off_values() != REF_SeCsr_int_off_values) {
        std::printf("SeCsr offsets %ld %ld %ld\n", p.off_starts(), p.off_idxs(), p.off_values());
        bad = 1;
    }
    const SeCsr<int>& c = p;
    const int sizes[] = REF_CSR_ROW_SIZE;
    const long offs[] = REF_CSR_IDXPTR_OFFSET;
    if (c.Rows() != REF_CSR_ROWS || c.Size() != REF_CSR_SIZE) bad = 1;
    for (int r = 0; r < REF_CSR_ROWS; ++r)
        if (c.Size(r) != sizes[r] || (long)(c.IdxPtr(r) - c.IdxPtr(0)) != offs[r]) {
            std::printf("SeCsr row %d\n", r);
            bad = 1;
        }
    if (c.Ptr() != &c) bad = 1;
    if (!bad) std::printf("layouts match the reference\n");
    return bad;
}
