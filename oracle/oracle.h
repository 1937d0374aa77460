/* oracle.h — TEST INFRASTRUCTURE ONLY. CPU restatement of the LeGO-LOAM-SR hot path used as
 * the parity checker (tests/, __graft_entry__.smoke) and as bench.py's cpu_baseline leg.
 * Never linked into the product library (lego-loam-sr_amd/).
 *
 * Parity status: the reference cannot be built here (ROS2/PCL/Eigen/GTSAM absent, SURVEY.md
 * §8c) and holds no golden vectors for this path, so this restatement is "parity unpinned"
 * against the reference binary. What IS pinned: its libm calls are host glibc, and the device
 * libm ports are checked bit-exactly against that glibc (libm_check.cpp); its kNN is checked
 * against the reference's vendored nanoflann.hpp compiled by path (oracle/Makefile, _ref/).
 */
#ifndef LLSR_ORACLE_H_
#define LLSR_ORACLE_H_
#include "../include/llsr.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_state oracle_state;

oracle_state* oracle_create(const llsr_config* cfg);
void oracle_destroy(oracle_state* s);
/* Reset the FA carry-over arrays (FA:167-198) to their value-initialised state. */
void oracle_reset(oracle_state* s);
/* One scan through ImageProjection::cloudHandler (IP:189-222) and the FeatureAssociation
 * feature stage (FA:2766-2775). Same output layout/semantics as llsr_process_scan. */
int32_t oracle_process_scan(oracle_state* s, const float* xyzi, int32_t n, llsr_scan_out* out);
/* The less-flat VoxelGrid's summation order (FA:1268-1270): pcl != 0 follows PCL (std::sort's
 * order of equal voxel ids, LLSR_VOXEL_ORDER_PCL), 0 sums in input order (LLSR_VOXEL_ORDER_INPUT,
 * the default of both sides). */
void oracle_set_voxel_order(oracle_state* s, int32_t pcl);
/* Per-stage wall time of the last oracle_process_scan (ms): IP, FA-features. */
void oracle_stage_ms(const oracle_state* s, double* ip_ms, double* fa_ms);
/* RANSAC with a caller seed (seed 12345 = PCL default) over the last scan's near-ground cloud;
 * used to show the synthetic scenes' inlier sets do not depend on the RNG. */
int32_t oracle_ransac_inliers(oracle_state* s, uint32_t seed, int32_t* inliers, int32_t cap);

/* MapOptimization::scan2MapOptimization (MO:1572-1610) on explicit inputs: corner queries
 * (laserCloudCornerScanDS), surf queries (laserCloudSurfTotalLastDS), corner / surf local maps
 * (…FromMapDS), float4 x,y,z,intensity each; `pose` = transformTobeMapped in/out.
 * cfg->mode selects faithful (update commented out, MO:1539-1545) or lm_applied. */
int32_t oracle_scan2map(const llsr_config* cfg, const float* corner_q, int32_t Qc, const float* surf_q,
                        int32_t Qs, const float* corner_map, int32_t Mc, const float* surf_map, int32_t Ms,
                        float* pose, llsr_lm_report* rep);
/* kNN-5 (d^2 < 1.0 accepted) of Q float4 queries in a float4 map: idx/d2 [Q][5], -1 = rejected.
 * liboracle: the 1 m grid; oracle/_ref/libref_mo.so exports the same as ref_knn5_batch /
 * ref_scan2map over the reference's nanoflann kd-tree. */
int32_t oracle_knn5_batch(const float* map, int32_t M, const float* q, int32_t Q, int32_t* idx, float* d2);
/* FeatureAssociation::updateTransformation (FA:2505-2535) on explicit clouds (see llsr.h).
 * transform_cur and is_degenerate are in/out (member state of the reference node). */
int32_t oracle_scan2scan(const llsr_config* cfg, const float* sharp, int32_t n_sharp, const float* flat,
                         int32_t n_flat, const float* corner_last, int32_t n_corner_last,
                         const float* surf_last, int32_t n_surf_last, float* transform_cur,
                         int32_t* is_degenerate, llsr_s2s_report* rep);
/* oracle_scan2map with the optimiser's members carried across calls (mapOptimization.h:279-281):
 * degenerate / matP[36] (column-major) in/out, as one MapOptimization instance over a sequence. */
int32_t oracle_scan2map_carry(const llsr_config* cfg, const float* corner_q, int32_t Qc, const float* surf_q,
                              int32_t Qs, const float* corner_map, int32_t Mc, const float* surf_map, int32_t Ms,
                              float* pose, int32_t* degenerate, float* matP, llsr_lm_report* rep);
/* MapOptimization::run's pose glue (oracle_mapping.cpp): publishOdometry -> OdometryToTransform
 * (FA:2612-2625, utility.h:99-113) and transformAssociateToMap (MO:458-581). */
void oracle_odometry_to_transform(const float* transform_sum_fa, float* transform_sum_mo);
void oracle_associate_to_map(const float* transform_sum, const float* transform_bef_mapped,
                             const float* transform_aft_mapped, float* transform_tobe_mapped,
                             float* transform_incre);
/* Split-correspondence scan-to-map with int64 fixed-point normal equations: the CPU statement of
 * llsr_scan2map_shard_* for one problem (see oracle_mo.cpp). partial() writes LLSR_NE_WORDS words
 * for rank/world; step() takes the words summed over every rank and returns 1 while active. */
typedef struct oracle_s2m_shard oracle_s2m_shard;
oracle_s2m_shard* oracle_s2m_shard_create(const llsr_config* cfg, const float* corner_q, int32_t Qc,
                                          const float* surf_q, int32_t Qs, const float* corner_map, int32_t Mc,
                                          const float* surf_map, int32_t Ms, const float* pose);
void oracle_s2m_shard_destroy(oracle_s2m_shard* s);
void oracle_s2m_shard_partial(oracle_s2m_shard* s, int32_t rank, int32_t world, int64_t* ne);
int32_t oracle_s2m_shard_step(oracle_s2m_shard* s, const int64_t* ne);
void oracle_s2m_shard_result(const oracle_s2m_shard* s, float* pose, llsr_lm_report* rep);
/* TransformToEnd (FA:1414-1490, no-IMU branch) of n float4 points in place. */
void oracle_transform_to_end(const float* transform_cur, float* xyzi, int32_t n);
/* integrateTransformation (FA:2537-2568, no IMU): transform_sum in place. */
void oracle_integrate_transformation(float* transform_sum, const float* transform_cur);
/* GenerateShadowPoint (FA:412-439). */
void oracle_shadow_points(float* out_xyzi);
/* Test hooks for the oracle's Eigen 3.3.7 restatement (oracle_eigen.h): column-major inputs. */
int32_t oracle_eig3(const float* A, float* evals, float* evecs);
int32_t oracle_eig6(const float* A, float* evals, float* evecs);
void oracle_qr_solve_5x3(const float* A, const float* b, float* x);
void oracle_qr_solve_6x6(const float* A, const float* b, float* x);

/* pcl::VoxelGrid<PointXYZI>::filter (oracle_voxel.h) of n float4 points; returns the centroid
 * count written to `out` (capacity n float4), -1 on bad arguments. stable != 0 sums each voxel in
 * input order (the device order) instead of the std::sort order. */
int64_t oracle_voxel_grid(const float* in, int64_t n, float leaf, int32_t stable, float* out);
/* Key poses (float4 x, y, z, intensity) with squared distance < float(radius^2) to pos, ascending
 * index (MO:1155-1159). _ref exports ref_keypose_radius over the reference's nanoflann. */
int32_t oracle_keypose_radius(const float* poses4, int32_t K, const float* pos, float radius, int32_t* out);
/* MapOptimization keyframe store + extractSurroundingKeyFrames (oracle_map.cpp). */
typedef struct oracle_map oracle_map;
oracle_map* oracle_map_create(float radius, float keypose_leaf, float corner_leaf, float surf_leaf,
                              int32_t loop_closure, int32_t search_num);
void oracle_map_destroy(oracle_map* m);
void oracle_transform_cloud(const float* pose6, const float* in, int64_t n, float* out);
int32_t oracle_map_add_keyframe(oracle_map* m, const float* pose6, const float* corner, int32_t n_corner,
                                const float* surf, int32_t n_surf, const float* outlier, int32_t n_outlier);
int32_t oracle_map_extract(oracle_map* m, const float* pos, int32_t stable, float* corner_out, int64_t cap_corner,
                           int64_t* n_corner, float* surf_out, int64_t cap_surf, int64_t* n_surf, int32_t* ids,
                           int32_t cap_ids, int32_t* n_ids, int64_t* raw_counts);

#ifdef __cplusplus
}
#endif
#endif
