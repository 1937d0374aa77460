/* llsr_rccl.h — multi-GPU scan-to-map over RCCL: the C++ host driver of the split-correspondence
 * mode (BASELINE.json configs[4]) for callers without Python — e.g. the
 * MapOptimization node of INTEGRATION.md §2 running one process per GPU.
 *
 * Library: lego-loam-sr_amd/libllsr_rccl.so (links libllsr.so and /opt/rocm/lib/librccl.so), kept
 * apart so that libllsr.so itself has no RCCL dependency. The reference loop it splits is
 * scan2MapOptimization's iteration loop (mapOptmization.cpp:1578-1608): per LM iteration, every rank
 * builds its share of the correspondences' normal equations, ONE ncclAllReduce (sum, int64) of the
 * [P][LLSR_NE_WORDS] words runs over xGMI, and every rank solves the same 6x6 systems — no
 * broadcast, and every rank stops after the same iteration because it holds the same sums.
 */
#ifndef LLSR_RCCL_H_
#define LLSR_RCCL_H_
#include <stdint.h>

#include "llsr.h"
#ifdef __cplusplus
extern "C" {
#endif

/* One split-correspondence scan-to-map batch on this rank (the handle must have been reserved as
 * for llsr_scan2map_batch; every rank passes the same batch):
 *   llsr_scan2map_shard_begin
 *   up to iterCountThres times (the handle's, llsr_get_config):
 *     llsr_scan2map_shard_partial(h, rank, world, d_ne)
 *     ncclAllReduce(d_ne, d_ne, P * LLSR_NE_WORDS, ncclInt64, ncclSum, comm, hip_stream)
 *     llsr_scan2map_shard_step(h, d_ne, n_active or NULL)   host check every `poll` iterations
 *   llsr_scan2map_shard_end
 * nccl_comm: an ncclComm_t of `world` ranks (ncclCommInitRank). hip_stream: the hipStream_t the
 * kernels and the collective share (required: NULL is LLSR_EINVAL, since RCCL would read it as the
 * legacy default stream, which is not ordered with the handle's own stream). d_ne: device int64
 * [P][LLSR_NE_WORDS] exchange buffer, or NULL to allocate one for the call. *iterations (may be
 * NULL) = LM iterations run (<= iterCountThres). The poses and reports land in batch->pose / batch->report,
 * bit-identical for every world size. LLSR_EIO when a collective fails (ncclGetLastError has the
 * text); the other codes as the llsr_scan2map_shard_* calls return them. */
int32_t llsr_scan2map_rccl(llsr_handle* h, const llsr_s2m_batch* batch, void* nccl_comm, int32_t rank,
                           int32_t world, int64_t* d_ne, int32_t poll, int32_t* iterations, void* hip_stream);

/* Mean wall time (us) of one ncclAllReduce of `words` int64 on hip_stream, synchronised per call,
 * over `reps` calls after 5 warm-up calls (d_words: device buffer of at least `words` int64). */
int32_t llsr_rccl_allreduce_us(void* nccl_comm, int64_t* d_words, int64_t words, int32_t reps, void* hip_stream,
                               float* us);

#ifdef __cplusplus
}
#endif
#endif /* LLSR_RCCL_H_ */
