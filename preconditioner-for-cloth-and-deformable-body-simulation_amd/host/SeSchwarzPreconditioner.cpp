// SeSchwarzPreconditioner.cpp -- the reference C++ surface
// (SeSchwarzPreconditioner.h:37-178) as a thin facade over the C ABI.
// Every method forwards to one mas_* call; see include/mas_capi.h for the
// mapping and the memory layouts.
#include "SeSchwarzPreconditioner.h"

#include <cstdio>
#include <cstring>
#include <string>

int CPU_THREAD_NUM = 1;  // SeOmp.cpp:29-33; the GPU path has no CPU threads

namespace SE {

SeSchwarzPreconditioner::SeSchwarzPreconditioner() {
    mas_config cfg{};
    cfg.device = -1;
    Check(mas_create(&m_handle, &cfg), "mas_create");
}

SeSchwarzPreconditioner::SeSchwarzPreconditioner(const mas_config& cfg) {
    Check(mas_create(&m_handle, &cfg), "mas_create");
}

SeSchwarzPreconditioner::~SeSchwarzPreconditioner() {
    if (m_handle) mas_destroy(m_handle);
}

void SeSchwarzPreconditioner::Check(int rc, const char* what) const {
    if (rc == MAS_OK) return;
    std::string msg = std::string("SeSchwarzPreconditioner: ") + what + " failed (" + std::to_string(rc) + ")";
    if (m_handle) msg += std::string(": ") + mas_last_error(m_handle);
    throw std::runtime_error(msg);
}

void SeSchwarzPreconditioner::AllocatePrecoditioner(int numVerts, int numEdges, int numFaces) {
    if (!m_positions || !m_neighbours) Check(MAS_ERR_ARG, "AllocatePrecoditioner (m_positions/m_neighbours unset)");
    m_numVerts = numVerts;
    Check(mas_allocate(m_handle, numVerts, numEdges, numFaces, &m_positions[0].x, m_neighbours->StartPtr(0),
                       m_neighbours->IdxPtr(0), m_edges ? m_edges[0].m_data : nullptr,
                       m_faces ? m_faces[0].m_data : nullptr),
          "AllocatePrecoditioner");
}

void SeSchwarzPreconditioner::PreparePreconditioner(const SeMatrix3f* diagonal, const SeMatrix3f* csrOffDiagonals,
                                                    const int* csrRanges, const EfSet* efSets, const EeSet* eeSets,
                                                    const VfSet* vfSets, unsigned int* efCounts,
                                                    unsigned int* eeCounts, unsigned int* vfCounts) {
    Check(mas_prepare(m_handle, diagonal->m_data, csrOffDiagonals->m_data, csrRanges, efSets, eeSets, vfSets,
                      efCounts, eeCounts, vfCounts),
          "PreparePreconditioner");
    // a non-SPD pivot (mas_config.strict_spd = 0): keep going as the reference
    // does (its method is void), but say so
    const char* w = mas_last_error(m_handle);
    if (w && std::strncmp(w, "warning:", 8) == 0) std::fprintf(stderr, "SeSchwarzPreconditioner: %s\n", w);
}

void SeSchwarzPreconditioner::Preconditioning(SeVec3fSimd* z, const SeVec3fSimd* residual, int /*dim*/) {
    Check(mas_apply(m_handle, &z[0].x, &residual[0].x), "Preconditioning");
}

void SeSchwarzPreconditioner::PreconditioningDevice(SeVec3fSimd* z, const SeVec3fSimd* residual, void* stream) {
    Check(mas_apply_device(m_handle, reinterpret_cast<float*>(z), reinterpret_cast<const float*>(residual), stream),
          "PreconditioningDevice");
}

}  // namespace SE
