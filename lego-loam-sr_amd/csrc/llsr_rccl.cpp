// llsr_rccl.cpp — libllsr_rccl.so: the C++ multi-GPU driver of the split-correspondence
// scan-to-map (include/llsr_rccl.h). Host code only: the per-iteration sequence of
// scan2MapOptimization's loop (mapOptmization.cpp:1578-1608) split at the normal equations,
// partial (this rank's query blocks) -> ncclAllReduce over xGMI -> solve, on one HIP stream so the
// kernels and the collective are ordered without host synchronisation (the host only reads the
// active-problem count every `poll` iterations).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdint>

#include "../../include/llsr.h"
#include "../../include/llsr_rccl.h"

namespace {

struct DeviceBuf {  // an exchange buffer allocated for one call (d_ne == NULL)
  int64_t* p = nullptr;
  ~DeviceBuf() {
    if (p) (void)hipFree(p);
  }
};

}  // namespace

extern "C" int32_t llsr_scan2map_rccl(llsr_handle* h, const llsr_s2m_batch* batch, void* nccl_comm, int32_t rank,
                                      int32_t world, int64_t* d_ne, int32_t poll, int32_t* iterations,
                                      void* hip_stream) {
  if (!h || !batch || !nccl_comm || !hip_stream || world < 1 || rank < 0 || rank >= world || batch->n_problems < 1)
    return LLSR_EINVAL;
  const int P = batch->n_problems;
  const size_t words = (size_t)P * LLSR_NE_WORDS;
  DeviceBuf own;
  if (!d_ne) {
    if (hipMalloc(&own.p, words * sizeof(int64_t)) != hipSuccess) return LLSR_ENOMEM;
    d_ne = own.p;
  }
  if (poll < 1) poll = 1;
  llsr_config cfg;
  if (llsr_get_config(h, &cfg) != LLSR_OK) return LLSR_EINVAL;
  const int iter_max = cfg.iterCountThres;  // the loop bound of MO:1578
  if (iter_max < 1) return LLSR_EINVAL;
  ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  int32_t rc = llsr_scan2map_shard_begin(h, batch, hip_stream);
  if (rc != LLSR_OK) return rc;
  // at most iterCountThres rounds (MO:1578); the host reads the active count every `poll` rounds
  // and on the last one, so a converged batch stops within poll - 1 rounds and never runs past
  // the bound when poll does not divide it (the device also marks every problem done there)
  int it = 0;
  while (it < iter_max) {
    rc = llsr_scan2map_shard_partial(h, rank, world, d_ne, hip_stream);
    if (rc != LLSR_OK) return rc;
    const ncclResult_t nr = ncclAllReduce(d_ne, d_ne, words, ncclInt64, ncclSum, comm, s);
    if (nr != ncclSuccess) return LLSR_EIO;
    ++it;
    int32_t active = -1;
    const bool check = it % poll == 0 || it == iter_max;
    rc = llsr_scan2map_shard_step(h, d_ne, check ? &active : nullptr, hip_stream);
    if (rc != LLSR_OK) return rc;
    if (active == 0) break;
  }
  rc = llsr_scan2map_shard_end(h, hip_stream);
  if (rc != LLSR_OK) return rc;
  if (iterations) *iterations = it;
  return LLSR_OK;
}

extern "C" int32_t llsr_rccl_allreduce_us(void* nccl_comm, int64_t* d_words, int64_t words, int32_t reps,
                                          void* hip_stream, float* us) {
  if (!nccl_comm || !d_words || words < 1 || reps < 1 || !us || !hip_stream) return LLSR_EINVAL;
  ncclComm_t comm = static_cast<ncclComm_t>(nccl_comm);
  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  auto once = [&]() {
    return ncclAllReduce(d_words, d_words, (size_t)words, ncclInt64, ncclSum, comm, s) == ncclSuccess &&
           hipStreamSynchronize(s) == hipSuccess;
  };
  for (int k = 0; k < 5; ++k)
    if (!once()) return LLSR_EIO;
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; ++k)
    if (!once()) return LLSR_EIO;
  const auto t1 = std::chrono::steady_clock::now();
  *us = (float)(std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
  return LLSR_OK;
}
