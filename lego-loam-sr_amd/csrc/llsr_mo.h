// llsr_mo.h — device data of the scan-to-map batch (llsr_mo.hip), shared with the host side.
#pragma once
#include <stdint.h>

#include "../../include/llsr.h"
#include "llsr_grid.h"

namespace llsr {

// Per-problem optimiser state, resident in HBM for the whole batch.
struct S2MProb {
  int64_t qc0, qs0, mc0, ms0;  // offsets of this problem's clouds
  int Qc, Qs, Mc, Ms;
  float pose[6];               // transformTobeMapped
  float cR, sR, cP, sP, cY, sY;  // cos/sin of pose[0..2] (MO:591-604, MO:1445-1450)
  float matP[36];
  float matX0[6];
  float min_lambda, cf_mean;
  int iter, active, converged, degenerate, nc, ns;
  int pad_[2];
};

struct S2MArgs {
  int P;
  int applied;                 // LLSR_MODE_LM_APPLIED
  int iter_max;                // iterCountThres
  float step_size, stop_thres;
  int cap_qc, cap_qs, cap_mc, cap_ms;
  int blocks_c;                // query blocks per problem reserved for corners (rest: surf)
  int blocks;                  // query blocks per problem (grid.x of k_s2m_iter)
  const float* cq; const int64_t* cq_off;
  const float* sq; const int64_t* sq_off;
  const float* cm; const int64_t* cm_off;
  const float* sm; const int64_t* sm_off;
  float* pose;                 // [P][6] in/out
  llsr_lm_report* report;      // [P]
  S2MProb* prob;               // [P]
  CellGrids2 grids;            // g[0] corner map, g[1] surf map
  float4* rows;                // [P][blocks][256][2] compacted matA rows per query block
  int* bcnt;                   // [P][blocks] rows per query block
  int* n_active;               // problems still iterating
  int* error;                  // capacity / offset violations
  // split-correspondence mode (llsr_scan2map_shard_*): this rank's share of the query blocks
  int rank, world;
  long long* ne;               // [P][llsr_lm::kNeWords] int64 fixed-point sums
  // MapOptimization members that outlive a frame (mapOptimization.h:279-281, zeroed at
  // construction MO:285-286): isDegenerate / matP in at setup and out at finish (mapping chain;
  // null: a fresh optimiser per problem)
  int solve_rows;              // matA rows k_s2m_solve stages in LDS at a time
  float* blk_spill;            // [P][spill_cap][29] Eigen depth-block sums beyond the 64 kept in LDS
  int spill_cap;               // depth blocks per problem in blk_spill
  int dbg;                     // diagnostics (LLSR_S2M_DBG): k_s2m_solve stops after stage dbg (0: never)
  const int* deg_in; const float* matP_in;
  int* deg_out; float* matP_out;
};

__global__ void k_s2m_setup(S2MArgs a);
__global__ void k_s2m_iter(S2MArgs a);

__global__ void k_s2m_solve(S2MArgs a);
constexpr int kSolveLds = 144 * 1024;  // k_s2m_solve's dynamic LDS (gfx950: 160 KB per workgroup)
__global__ void k_s2m_finish(S2MArgs a);
__global__ void k_s2m_iter_fx(S2MArgs a, int nb);
__global__ void k_s2m_solve_fx(S2MArgs a);

}  // namespace llsr
