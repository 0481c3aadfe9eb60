// Compile-time check that the facade keeps the reference's memory layouts
// (SeVectorSimd.h:45-57, SeMatrix.h:650-682, SeCollisionElements.h:33-58).
#include <cstddef>

#include "SeSchwarzPreconditioner.h"

using namespace SE;
static_assert(sizeof(SeVec3fSimd) == 16 && alignof(SeVec3fSimd) == 16, "SeVec3fSimd");
static_assert(sizeof(SeMatrix3f) == 36, "SeMatrix3f");
static_assert(sizeof(Int4) == 16 && alignof(Int4) == 16, "Int4");
static_assert(sizeof(Float2) == 8 && alignof(Float2) == 8, "Float2");
static_assert(sizeof(Float3) == 12, "Float3");
static_assert(offsetof(EfSet, m_eId) == 0 && offsetof(EfSet, m_fId) == 4 && offsetof(EfSet, stiff) == 8 &&
                  offsetof(EfSet, m_bary) == 12 && offsetof(EfSet, m_normal) == 32 && sizeof(EfSet) == 48,
              "EfSet");
static_assert(offsetof(VfSet, m_bary) == 16 && offsetof(VfSet, m_normal) == 32 && sizeof(VfSet) == 48, "VfSet");
static_assert(offsetof(EeSet, m_bary) == 16 && offsetof(EeSet, m_normal) == 32 && sizeof(EeSet) == 48, "EeSet");

int main() {
    SeMatrix3f m = SeMatrix3f::Identity();
    m(0, 1) = 2.f;  // column-major: element (0,1) lives at m_data[3]
    return m.m_data[3] == 2.f ? 0 : 1;
}
