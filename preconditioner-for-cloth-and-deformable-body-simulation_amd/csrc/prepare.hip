// prepare.hip -- PreparePreconditioner orchestration (.cpp:67-98):
// stencils -> aggregation levels -> block assembly -> batched factor -> apply tables.
#include "mas_internal.h"

namespace mas {

int prepare_apply_tables(mas_context* h, hipStream_t s);

int finish_early(mas_context* h) {
    if (!h->earlyPending) return MAS_OK;
    h->prepWorker->wait();
    h->earlyPending = false;
    return h->earlyRc ? fail(h, h->earlyRc, h->earlyErr) : MAS_OK;
}

int run_prepare(mas_context* h, const float* d_diag9, const float* d_off9, const int* d_ranges, const void* ef,
                const void* ee, const void* vf, const unsigned* efC, const unsigned* eeC, const unsigned* vfC,
                hipStream_t s) {
    int rc;
    h->prepared = false;
    h->err.clear();  // after a successful Prepare: empty, or the non-SPD warning
    // a previous Prepare that failed between the side fold's fork and join
    // (run_assemble) may have left it running: this Prepare's memsets wait
    if (h->foldStream) {
        hipStreamWaitEvent(s, h->evFoldJoin, 0);
        if (h->preFactored) hipStreamWaitEvent(s, h->evPreJoin, 0);
    }
    h->preFactored = false;
    hipEventRecord(h->ev[2], s);
    // pivot checks of this Prepare's factors: [0] count, [1] lowest block (k_factor.hip check_pivots)
    int* status = P<int>(h->devStatus);
    if ((rc = hip_check(h, hipMemsetD32Async(status, 0, 1, s), "status")) ||
        (rc = hip_check(h, hipMemsetD32Async(status + 1, 0x7fffffff, 1, s), "status")))
        return rc;
    if ((rc = build_stencils(h, ef, ee, vf, efC, eeC, vfC, s))) return rc;
    ScopedEvents ev;
    if (!ev.ok()) return fail(h, MAS_ERR_HIP, "hipEventCreate");
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1];
    // the level-0 blocks this Prepare assembles and factors: all, or those of
    // the Morton shard set by mas_set_prepare_shard (mas_shard_plan's split);
    // level 0 is the sorted vertices, known before the levels are built
    h->nFineBlk = ceil32(h->nV) / 32;
    h->fineBlk0 = (int)((long long)h->prepRank * h->nFineBlk / h->prepWorld);
    h->fineBlk1 = (int)((long long)(h->prepRank + 1) * h->nFineBlk / h->prepWorld);
    // fused variants: the level-0 contacts and the fused kernel start on
    // prepStream after the stencils (the fork event), beside the level build;
    // their launches are queued while the level kernels run (run_levels' hook)
    h->earlyFused = false;
    h->nBlkPrev = h->nBlk;
    const bool early = early_fused_wanted(h);
    h->earlyPlanned = early;
    if (early && ((rc = prep_stream_init(h)) || (rc = hip_check(h, hipEventRecord(h->evPrepFork, s), "fork"))))
        return rc;
    // buffers both threads use (the worker writes inv, add0 and, early_od,
    // od and the record counts; this thread's assembly reads them) are sized
    // here, before the worker starts: ensure() on one Buffer from two threads
    // could allocate it twice and leave them with different pointers
    if (early && (rc = early_buffers(h))) return rc;
    // the worker's job never outlives this call, whatever path returns
    // (on an error return of this thread: joined without reporting, so
    // mas_last_error keeps this thread's message, not the worker's)
    struct JoinEarly {
        mas_context* h;
        ~JoinEarly() {
            if (!h->earlyPending) return;
            h->prepWorker->wait();
            h->earlyPending = false;
        }
    } joinEarly{h};
    if (early && h->earlyThread) {
        // a second host thread queues prepStream's work while this one queues
        // the level build and the coarse assembly: each stream is fed from
        // the start (one thread queueing both left the early path behind the
        // level kernels): the handle's PrepWorker, which selects the handle's
        // device first (ensure() allocates on the current device).  This
        // thread waits for it only where it needs the early path's state
        // (finish_early in run_assemble): waiting right after the level build
        // kept the coarse assembly ~300 us behind the worker's ~40 launches.
        if (!h->prepWorker) h->prepWorker = std::make_unique<PrepWorker>(h->device);
        h->earlyRc = MAS_OK;
        h->earlyErr.clear();
        h->earlyPending = true;
        h->prepWorker->post([h, d_diag9, d_off9, d_ranges, s](bool devOk) {
            if (!devOk) {
                h->earlyRc = MAS_ERR_HIP;
                h->earlyErr = "early Prepare thread: hipSetDevice failed";
                return;
            }
            ErrorSink sink(&h->earlyErr);  // fail() from this thread writes earlyErr, not h->err
            h->earlyRc = run_level0_early(h, d_diag9, d_off9, d_ranges, s);
        });
        if ((rc = run_levels(h, s, d_ranges))) return rc;
    } else if ((rc = run_levels(h, s, d_ranges, [&]() {
                    return early ? run_level0_early(h, d_diag9, d_off9, d_ranges, s) : MAS_OK;
                }))) {
        return rc;
    }
    if (h->fusedAfterLevels && ((rc = finish_early(h)) || (h->earlyFused && (rc = launch_level0_fused(h, s)))))
        return rc;
    // a sharded Prepare: which coarse rows this rank assembles (coarse_split.hip)
    if ((rc = plan_coarse_split(h, s))) return rc;
    hipEventRecord(e0, s);
    if ((rc = run_assemble(h, d_diag9, d_off9, d_ranges, s)) || (rc = finish_early(h))) return rc;
    hipEventRecord(e1, s);
    if ((rc = run_factor(h, s))) return rc;
    // the coarse rows other ranks need; exchanged here when the handle has a
    // communicator of this shard or an allgather hook, else by the caller
    // (mas_prepare_shard_rows / mas_prepare_shard_complete)
    if (h->splitPlanned) {
        if ((rc = pack_coarse_rows(h, s))) return rc;
        const bool viaRccl = h->rcclComm && h->rcclRank == h->prepRank && h->rcclWorld == h->prepWorld;
        if (viaRccl || h->prepAllgather) {
            const size_t segBytes = (size_t)h->splitSegRows * 1152;
            if ((rc = ensure(h, h->prepGathered, segBytes * h->prepWorld))) return rc;
            if (viaRccl) {
                if ((rc = comm_allgather(h, h->prepSeg.p, h->prepGathered.p, segBytes, s))) return rc;
            } else if (int e = h->prepAllgather(h->prepSeg.p, h->prepGathered.p, segBytes, s, h->prepAllgatherUser)) {
                return fail(h, MAS_ERR_COMM, "Prepare's allgather hook returned " + std::to_string(e));
            }
            if ((rc = complete_coarse_rows(h, P<float>(h->prepGathered), s))) return rc;
        }
    }
    const int nCoarseNodes = h->totalClusters - h->levelSize[3];
    if ((rc = ensure(h, h->Rc, (size_t)(nCoarseNodes > 0 ? nCoarseNodes : 1) * 16)) ||
        (rc = ensure(h, h->Zc, (size_t)(nCoarseNodes > 0 ? nCoarseNodes : 1) * 16)))
        return rc;
    // Zc too: mas_profile_fine prolongs from it before the first apply has written it
    if (nCoarseNodes > 0 &&
        ((rc = hip_check(h, hipMemsetAsync(h->Rc.p, 0, (size_t)nCoarseNodes * 16, s), "memset Rc")) ||
         (rc = hip_check(h, hipMemsetAsync(h->Zc.p, 0, (size_t)nCoarseNodes * 16, s), "memset Zc"))))
        return rc;
    // the apply tables depend on the hierarchy alone: kept while it is unchanged
    if (!h->hierCache || h->tabHierId != h->hierId) {
        h->tabHierId = ~0ull;
        if ((rc = prepare_apply_tables(h, s))) return rc;
        h->tabHierId = h->hierId;
        h->l1First.clear();  // per-bank level-1 starts: computed on first use (sharding, blob save)
        h->shardWorld = 0;
    }
    // the side stream's level-1 factor (coarse split) and the fused level-0
    // kernel (prepStream) join last: nothing above needs their inverses
    if (h->preFactored && (rc = hip_check(h, hipStreamWaitEvent(s, h->evPreJoin, 0), "join pre factor"))) return rc;
    if (h->factorVariant >= 4 && (rc = hip_check(h, hipStreamWaitEvent(s, h->evPrepJoin, 0), "join fused factor")))
        return rc;
    hipEventRecord(h->ev[3], s);
    if ((rc = hip_check(h, hipStreamSynchronize(s), "prepare sync"))) return rc;
    float a = 0, b = 0, c = 0, t = 0;
    hipEventElapsedTime(&t, h->ev[2], h->ev[3]);
    hipEventElapsedTime(&a, h->ev[2], e0);
    hipEventElapsedTime(&b, e0, e1);
    hipEventElapsedTime(&c, e1, h->ev[3]);
    h->stats.prepare_ms = t;
    h->stats.prepare_levels_ms = a;
    h->stats.prepare_assemble_ms = b;
    h->stats.prepare_factor_ms = c;
    float f = 0, f0 = 0;
    if (h->factorVariant >= 4 && h->evFine[0]) {
        hipEventElapsedTime(&f, h->evFine[0], h->evFine[1]);
        hipEventElapsedTime(&f0, h->ev[2], h->evFine[0]);
    }
    h->stats.prepare_fine_ms = f;
    h->stats.prepare_fine_start_ms = f0;
    h->stats.factor_formation = (h->factorVariant == 5 || h->factorVariant == 3) ? 1 : 0;
    h->stats.hier_dirty_level = h->hierCache ? h->lastHierDirty : -1;
    h->stats.hier_rebuilt = h->lastHierBuilt ? 1 : 0;
    h->stats.coarse_split = h->splitPlanned ? (h->splitClean ? 1 : 2) : 0;
    h->prepared = true;  // as the reference: the inverses exist (with the bad pivots in them)
    return report_pivots(h, s);
}

int report_pivots(mas_context* h, hipStream_t s) {
    int* status = P<int>(h->devStatus);
    int bad[2] = {0, 0};
    int rc;
    if ((rc = read_back(h, s, {status, status + 1}, bad))) return rc;
    h->stats.nonspd_blocks = bad[0];
    if (bad[0] > 0) {
        int level = 0;
        for (int l = 1; l < h->L; ++l)
            if (32 * bad[1] >= h->levelSize[2 * l + 1]) level = l;
        const std::string msg = std::to_string(bad[0]) + " block(s) met a zero, negative or non-finite pivot in "
                                "LDL^T (first: block " + std::to_string(bad[1]) + ", level " + std::to_string(level) +
                                "): the Hessian is not SPD there; the reference divides by it unchecked "
                                "(.cpp:1406,1431)";
        // strict_spd: fail; else keep going as the reference does, with a warning
        if (h->cfg.strict_spd) return fail(h, MAS_ERR_NOT_SPD, msg);
        fail(h, MAS_OK, "warning: " + msg);
    }
    return MAS_OK;
}

}  // namespace mas
