// SeSchwarzPreconditioner.h -- drop-in C++ surface of the reference
// (V-Sekai/preconditioner-for-cloth-and-deformable-body-simulation,
// SeSchwarzPreconditioner.h:37-178), backed by the MI355X C ABI (mas_capi.h).
//
// Same namespace (SE), class name, public members and method signatures --
// including the reference's spelling of AllocatePrecoditioner -- and
// layout-compatible value types, so a PCG loop written against the reference
// compiles and links against libSeSchwarzPreconditioner.so unchanged:
//
//   SeVec3fSimd  16 B, 16-aligned {x,y,z,w}        SeVectorSimd.h:45-57
//   SeMatrix3f   9 floats, column-major m(i,j)=[j*3+i] SeMatrix.h:650-682
//   Int4         4 ints, 16-aligned                 SeVector.h:270,395
//   Float2/3     8-aligned pair / packed triple     SeVector.h:162,215
//   EfSet/VfSet/EeSet 48-byte contact records       SeCollisionElements.h:33-58
//   SeCsr<int>   Size(id), IdxPtr(id), StartPtr(id) SeCsr.h:119-173
//
// The methods are void like the reference's; a failure throws
// std::runtime_error carrying mas_last_error() (the reference has no error
// channel at all).  Not thread-safe (neither is the reference).
#pragma once

#include <cstddef>
#include <stdexcept>
#include <vector>

#include "mas_capi.h"

extern int CPU_THREAD_NUM;  // SeOmp.cpp:29-33 (link compatibility; unused by the GPU path)

namespace SE {

struct alignas(16) SeVec3fSimd {
    float x, y, z, w;
    SeVec3fSimd() {}
    explicit SeVec3fSimd(float s) : x(s), y(s), z(s), w(0.f) {}
    SeVec3fSimd(float a, float b, float c) : x(a), y(b), z(c), w(0.f) {}
    SeVec3fSimd(float a, float b, float c, float d) : x(a), y(b), z(c), w(d) {}
    float& operator[](unsigned i) { return (&x)[i]; }
    const float& operator[](unsigned i) const { return (&x)[i]; }
};
using Simd3f = SeVec3fSimd;

class SeMatrix3f {
  public:
    SeMatrix3f() {}
    explicit SeMatrix3f(float v) {
        for (float& d : m_data) d = v;
    }
    float& operator()(int i, int j) { return m_data[j * 3 + i]; }
    const float& operator()(int i, int j) const { return m_data[j * 3 + i]; }
    static SeMatrix3f Identity() {
        SeMatrix3f m(0.f);
        m(0, 0) = m(1, 1) = m(2, 2) = 1.f;
        return m;
    }
    float m_data[9];
};

struct alignas(16) Int4 {
    int m_data[4];
    int& operator[](unsigned i) { return m_data[i]; }
    const int& operator[](unsigned i) const { return m_data[i]; }
};
struct alignas(8) Float2 {
    float values[2];
    float& operator[](unsigned i) { return values[i]; }
    const float& operator[](unsigned i) const { return values[i]; }
};
struct Float3 {
    float values[3];
    float& operator[](unsigned i) { return values[i]; }
    const float& operator[](unsigned i) const { return values[i]; }
};

struct EfSet {
    int m_eId;
    int m_fId;
    float stiff;
    Float3 m_bary;
    SeVec3fSimd m_normal;
};
struct VfSet {
    int m_vId;
    int m_fId;
    float stiff;
    Float2 m_bary;
    SeVec3fSimd m_normal;
};
struct EeSet {
    int m_eId0;
    int m_eId1;
    float stiff;
    Float2 m_bary;
    SeVec3fSimd m_normal;
};
static_assert(sizeof(SeVec3fSimd) == 16 && sizeof(SeMatrix3f) == 36 && sizeof(Int4) == 16, "layout");
static_assert(sizeof(EfSet) == 48 && sizeof(VfSet) == 48 && sizeof(EeSet) == 48, "contact record layout");
static_assert(offsetof(EfSet, m_bary) == 12 && offsetof(VfSet, m_bary) == 16 && offsetof(EfSet, m_normal) == 32,
              "contact record layout");

// SeCompressSparseData<Type> / SeCsr<Type> (SeCsr.h:35-173): rows m_starts[n+1],
// column ids m_idxs.  Same object layout as the reference's class (vtable
// pointer, then the three vectors; 80 B for SeCsr<int> with libstdc++), pinned
// against the reference's own header by tests/test_ref_pinned.py.
template <typename Type>
class SeCompressSparseData {
  public:
    SeCompressSparseData() {}
    SeCompressSparseData(const std::vector<int>& starts, const std::vector<int>& idxs,
                         const std::vector<Type>& values)
        : m_starts(starts), m_idxs(idxs), m_values(values) {}
    virtual ~SeCompressSparseData() {}
    int Size() const { return m_starts.back(); }
    int Size(int id) const { return m_starts[id + 1] - m_starts[id]; }
    int Start(int id) const { return m_starts[id]; }
    const int* StartPtr(int id) const { return &m_starts[id]; }
    int Idx(int id) const { return m_idxs[id]; }
    const int* IdxPtr(int id) const { return m_idxs.data() + m_starts[id]; }
    const Type* ValuePtr(int id) const { return m_values.data() + m_starts[id]; }
    virtual const SeCompressSparseData* Ptr() const { return this; }

  protected:
    std::vector<int> m_starts;
    std::vector<int> m_idxs;
    std::vector<Type> m_values;
};

template <typename Type>
class SeCsr : public SeCompressSparseData<Type> {
  public:
    SeCsr() {}
    SeCsr(const std::vector<int>& starts, const std::vector<int>& idxs, const std::vector<Type>& values)
        : SeCompressSparseData<Type>(starts, idxs, values) {}
    int Rows() const { return (int)SeCompressSparseData<Type>::m_starts.size() - 1; }
    const SeCsr* Ptr() const override { return this; }
};

class SeSchwarzPreconditioner {
  public:
    //==== input data (SeSchwarzPreconditioner.h:44-51), borrowed pointers
    const SeVec3fSimd* m_positions = nullptr;
    const Int4* m_edges = nullptr;
    const Int4* m_faces = nullptr;
    const SeCsr<int>* m_neighbours = nullptr;

    SeSchwarzPreconditioner();
    explicit SeSchwarzPreconditioner(const mas_config& cfg);
    ~SeSchwarzPreconditioner();
    SeSchwarzPreconditioner(const SeSchwarzPreconditioner&) = delete;
    SeSchwarzPreconditioner& operator=(const SeSchwarzPreconditioner&) = delete;

    //==== call before time integration once a frame (.h:56)
    void AllocatePrecoditioner(int numVerts, int numEdges, int numFaces);
    void AllocatePreconditioner(int numVerts, int numEdges, int numFaces) {
        AllocatePrecoditioner(numVerts, numEdges, numFaces);
    }

    //==== call before PCG iteration loop (.h:59-60)
    void PreparePreconditioner(const SeMatrix3f* diagonal, const SeMatrix3f* csrOffDiagonals, const int* csrRanges,
                               const EfSet* efSets, const EeSet* eeSets, const VfSet* vfSets, unsigned int* efCounts,
                               unsigned int* eeCounts, unsigned int* vfCounts);

    //==== call during PCG iterations (.h:63); dim is unused, as in the reference
    void Preconditioning(SeVec3fSimd* z, const SeVec3fSimd* residual, int dim);

    //==== MI355X extensions
    // z and residual are device pointers (hipMalloc'd float4[nV]); stream is a hipStream_t.
    void PreconditioningDevice(SeVec3fSimd* z, const SeVec3fSimd* residual, void* stream = nullptr);
    mas_handle Handle() const { return m_handle; }

  private:
    void Check(int rc, const char* what) const;
    mas_handle m_handle = nullptr;
    int m_numVerts = 0;
};

}  // namespace SE
