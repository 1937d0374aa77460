/* llsr.h — C-ABI of the MI355X-native LeGO-LOAM-SR per-scan hot path.
 *
 * Drop-in boundary for the reference's ImageProjection → FeatureAssociation handoff
 * (LeGO-LOAM/src/imageProjection.cpp:189-222 cloudHandler, featureAssociation.cpp:2742-2778
 * runFeatureAssociation feature stage; stage types utility.h:63-83, cloud_msgs/msg/CloudInfo.msg).
 * The reference has no FFI of its own; these entry points replace the arithmetic behind the
 * node callbacks so a ROS2 shim keeps every topic and the Channel semantics.
 *
 * Conventions: plain C types only; int status codes (0 = OK, negative errno-style);
 * llsr_last_error() gives text; no C++ exception crosses the ABI. A handle is single-threaded
 * (one per pipeline/stream), matching the reference's one-thread-per-node layout.
 * Caller owns every host buffer; device buffers live in the handle.
 */
#ifndef LLSR_H_
#define LLSR_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Bumped on every change of a struct layout or entry-point signature. Version 2: llsr_map_config
 * gained enable_loop_closure and surrounding_keyframe_search_num (5 floats -> 5 floats + 2 int32),
 * so a caller built against version 1 would pass a struct the library reads past. A consumer checks
 * llsr_abi_version() == LLSR_ABI_VERSION once after loading the library. */
#define LLSR_ABI_VERSION 2

/* LLSR_ABI_VERSION as compiled into the loaded library. */
int32_t llsr_abi_version(void);
/* 16 hex digits identifying the kernel sources the library was built from (a hash of them): the
 * performance records under profiles/ name the build they measured. */
const char* llsr_build_id(void);

#define LLSR_OK 0
#define LLSR_EINVAL (-22)
#define LLSR_ENOMEM (-12)
#define LLSR_ENODEV (-19)
#define LLSR_ERANGE (-34)
#define LLSR_ENOSYS (-38)
#define LLSR_EIO (-5)

#define LLSR_LIDAR_VLP16 0
#define LLSR_LIDAR_HDL64E 2

#define LLSR_MODE_FAITHFUL 0
#define LLSR_MODE_LM_APPLIED 1

/* Mirrors the ROS2 parameters of the three nodes (loam_config.yaml:1-67 / 137-203;
 * read at imageProjection.cpp:80-121, featureAssociation.cpp:112-154). Angles in degrees,
 * exactly as in the YAML; the library applies the reference's conversions. */
typedef struct llsr_config {
  int32_t num_vertical_scans;      /* laser.num_vertical_scans   (H)          */
  int32_t num_horizontal_scans;    /* laser.num_horizontal_scans (W)          */
  float vertical_angle_bottom;     /* deg */
  float vertical_angle_top;        /* deg */
  float sensor_mount_angle;        /* deg (read but unused by groundRemovalOurs) */
  int32_t ground_scan_index;
  int32_t use_kitti;               /* ground angle D = 60/25 deg by row (IP:561-566) */
  int32_t use_vlp32c;              /* must be 0: VLP-32c row-histogram branch is not built */
  float segment_theta;             /* deg */
  int32_t segment_valid_point_num;
  int32_t segment_valid_line_num;
  float scan_period;               /* s */
  float edge_threshold;
  float surf_threshold;
  float nearest_feature_search_distance;
  float DBFr;
  float RatioXY;
  float RatioZ;
  int32_t mapping_frequency_divider;
  int32_t iterCountThres;          /* map_optimization.mapping.iterCountThres */
  float step_size;
  float stop_thres;
  int32_t mode;                    /* LLSR_MODE_* */
} llsr_config;

/* Fill *cfg with the YAML block for `lidar` (LLSR_LIDAR_VLP16 / LLSR_LIDAR_HDL64E). */
int32_t llsr_config_default(llsr_config* cfg, int32_t lidar);

/* The less-flat VoxelGrid of the feature stage (surfPointsLessFlatScan, FA:1268-1270) averages
 * each 0.2 m voxel's points. PCL sums them in the order std::sort leaves its index_vector (equal
 * voxel ids in libstdc++ introsort's order); the default, LLSR_VOXEL_ORDER_PCL, reproduces that
 * exactly (each ring's workgroup runs the introsort, partitions level by level). The opt-in
 * LLSR_VOXEL_ORDER_INPUT sums each voxel in ring order instead (a centroid may differ from PCL's in
 * the last bits when its voxel holds three or more points; voxel set, count and order are the
 * same), and the difference reaches the next scan's laserCloudSurfLast and so every later pose.
 * MapOptimization's VoxelGrids (llsr_map_*, llsr_mapping_*) always follow PCL's order. */
#define LLSR_VOXEL_ORDER_INPUT 0
#define LLSR_VOXEL_ORDER_PCL 1

/* Per-scan outputs of projection+segmentation (IP) and feature extraction (FA), in the
 * reference's own order. Host buffers, caller-allocated; capacities from llsr_query_sizes().
 * Any pointer may be NULL to skip that output. Counts are always written. */
typedef struct llsr_scan_out {
  /* ---- ImageProjection (IP) ---- */
  int32_t n_points;            /* finite input points (after removeNaNFromPointCloud, IP:198) */
  float orientation[3];        /* start, end, diff (CloudInfo.msg:6-8; IP:430-445) */
  float* range_image;          /* [H*W] _range_mat, FLT_MAX where empty (IP:337)          */
  int32_t* cell_point;         /* [H*W] raw-input index of the point kept in the cell, -1  */
  int8_t* ground_image;        /* [H*W] _ground_mat after groundRemovalOurs (IP:522-774)  */
  int32_t* label_image;        /* [H*W] _label_mat after cloudSegmentation (IP:776-931)   */
  int32_t* start_ring_index;   /* [H] CloudInfo.start_ring_index (IP:794)                 */
  int32_t* end_ring_index;     /* [H] CloudInfo.end_ring_index   (IP:831)                 */
  int32_t n_segmented;         /* S */
  float* seg_xyzi;             /* [4*S] _segmented_cloud (intensity = row + col/1e4)      */
  uint8_t* seg_ground_flag;    /* [S] CloudInfo.segmented_cloud_ground_flag               */
  uint32_t* seg_col_ind;       /* [S] CloudInfo.segmented_cloud_col_ind                   */
  float* seg_range;            /* [S] CloudInfo.segmented_cloud_range                     */
  float* seg_intensity;        /* [S] ProjectionOut.segmentedCloud_Intensity              */
  int32_t n_outlier;           /* O */
  float* outlier_xyzi;         /* [4*O] _outlier_cloud                                    */
  float* outlier_intensity;    /* [O] ProjectionOut.outlierCloud_Intensity                */
  int32_t n_near;              /* nearground_cloud size K (IP:700-715)                    */
  int32_t n_ransac_inliers;    /* RANSAC inliers (IP:716-721)                             */
  int32_t ransac_iterations;   /* PCL iterations_ after computeModel                      */
  /* ---- FeatureAssociation feature stage (FA:2766-2775) ---- */
  float* loam_xyzi;            /* [4*S] segmentedCloud after adjustDistortion (FA:565-789) */
  float* curvature;            /* [S] cloudCurvature, defined on [5, S-5) (FA:817-848)     */
  uint8_t* picked;             /* [S] cloudNeighborPicked after extractFeaturesOurs         */
  int8_t* label;               /* [S] cloudLabel after extractFeaturesOurs                  */
  int32_t n_less_sharp;        /* M */
  int32_t* less_sharp_ind;     /* [M] cornerPointsLessSharp as segmented indices           */
  int32_t* dbscan_cluster;     /* [M] DBSCAN_EdgeFeature cluster labels (FA:1318-1387)      */
  int32_t n_sharp;
  int32_t* sharp_ind;          /* cornerPointsSharp as segmented indices (FA:1299-1305)     */
  int32_t n_flat;              /* surfPointsFlat WITHOUT the 160 shadow points               */
  int32_t* flat_ind;           /* segmented indices; shadow points follow implicitly         */
  int32_t n_less_flat;
  float* less_flat_xyzi;       /* [4*L] surfPointsLessFlat (per-ring VoxelGrid 0.2, FA:1268) */
} llsr_scan_out;

/* Result of one scan-to-map optimisation (MapOptimization::scan2MapOptimization, MO:1572-1610). */
typedef struct llsr_lm_report {
  int32_t iterations;     /* iter_num (MO:1581): 200 in faithful mode unless iteration 0 converges */
  int32_t converged;      /* LMOptimization returned true */
  int32_t degenerate;     /* isDegenerate (MO:1518-1529) */
  float min_lambda;       /* smallest eigenvalue of J^T J at iteration 0 (MO:1515) */
  float cf_mean;          /* mean |residual| of the last evaluated iteration (MO:1560/1568) */
  int32_t n_corner_corr;  /* corner / surf correspondences kept at the last iteration */
  int32_t n_surf_corr;
  float matX0[6];         /* the iteration-0 step matX (faithful-mode parity target) */
  float pose[6];          /* final transformTobeMapped */
  float ms;               /* wall/device time of the optimisation, ms */
} llsr_lm_report;

typedef struct llsr_sizes {
  int32_t cells;               /* H*W: bound for every per-point array */
  int32_t rings;               /* H */
  int32_t max_points;          /* input points per scan accepted by the handle */
  int32_t shadow_points;       /* 160 virtual points (FA:412-450) */
} llsr_sizes;

typedef struct llsr_handle llsr_handle;
/* The configuration a handle was created with (e.g. iterCountThres for a host loop that drives
 * the llsr_scan2map_shard_* steps itself). */
int32_t llsr_get_config(const llsr_handle* h, llsr_config* cfg);

/* Create a handle on HIP device `hip_device` able to process batches of up to `max_batch`
 * scans of up to `max_points` raw points each. Fails with LLSR_ENODEV when no device or the
 * HIP kernels are unavailable — there is no CPU fallback behind this ABI. */
int32_t llsr_create(const llsr_config* cfg, int32_t hip_device, int32_t max_batch,
                    int32_t max_points, llsr_handle** out);
void llsr_destroy(llsr_handle* h);
const char* llsr_last_error(const llsr_handle* h);
int32_t llsr_query_sizes(const llsr_handle* h, llsr_sizes* out);
/* Reset the per-slot FeatureAssociation carry-over state (FA:167-198: the H*W arrays that the
 * reference sizes once and never clears). */
int32_t llsr_reset_state(llsr_handle* h);
/* LLSR_VOXEL_ORDER_PCL (default) or LLSR_VOXEL_ORDER_INPUT for the less-flat VoxelGrid; takes
 * effect from the next batch. */
int32_t llsr_set_voxel_order(llsr_handle* h, int32_t order);

/* One scan, host buffers in/out: the ImageProjection::cloudHandler + FeatureAssociation
 * feature-stage replacement. `xyzi` holds n raw points (x,y,z,intensity, NaN allowed). */
int32_t llsr_process_scan(llsr_handle* h, const float* xyzi, int32_t n, llsr_scan_out* out);

/* Batched, device-resident: scans b = 0..B-1 are d_xyzi[d_offsets[b] .. d_offsets[b+1]),
 * float4 records in HBM (B+1 int64 offsets, also in device memory). Slot b uses FA carry-over
 * state b. Enqueued on `hip_stream` (hipStream_t); NULL selects the handle's own stream, which is
 * created non-blocking — it does NOT synchronise with the legacy default stream, so a caller that
 * filled d_xyzi on the default stream must pass that stream (or synchronise) itself. Returns after
 * enqueue. Batches of one handle are ordered even across streams (each waits for the previous
 * one's completion event), because they share the slot buffers and the FA carry-over state.
 * d_xyzi and d_offsets must stay valid and unchanged until the batch has completed: the kernels
 * read them while they run.
 * Results stay in the handle until the next call. */
int32_t llsr_process_batch(llsr_handle* h, const float* d_xyzi, const int64_t* d_offsets,
                           int32_t B, void* hip_stream);

/* Copy slot b's results of the last batch into host buffers (synchronises the stream). */
int32_t llsr_fetch_scan(llsr_handle* h, int32_t b, llsr_scan_out* out);

/* ImageProjection's visualization topics for slot b of the last batch (publishClouds,
 * imageProjection.cpp:933-967), built on the device from the slot's range image, kept points,
 * ground and label images, then copied to the caller's host buffers (each may be NULL: skipped):
 *   full_cloud / full_info_cloud  [H*W][4]  /full_cloud (IP:54), /full_cloud_info: per cell
 *       x, y, z with intensity row + col / 1e4 resp. the range (IP:337-347); resetParameters'
 *       nanPoint (NaN x, y, z, intensity 0) where no point landed (IP:170-179)
 *   ground / nonground / unknownground_cloud  [<= H*W][4]  the full-cloud points of the cells
 *       whose final ground_mat is 1 / 0 / 2, row-major (IP:760-769)
 *   segmented_cloud_pure  [<= H*W][4]  cells with 0 < label != 999999, intensity = label,
 *       row-major (IP:833-842)
 * The n_* fields receive the four clouds' sizes. Synchronises. */
typedef struct llsr_vis_out {
  float* full_cloud;
  float* full_info_cloud;
  float* ground_cloud;
  float* nonground_cloud;
  float* unknownground_cloud;
  float* segmented_cloud_pure;
  int32_t n_ground;
  int32_t n_nonground;
  int32_t n_unknownground;
  int32_t n_segmented_pure;
} llsr_vis_out;
int32_t llsr_fetch_vis_clouds(llsr_handle* h, int32_t b, llsr_vis_out* out);

/* Device-side counters of the last batch: per slot {n_points, S, O, M, n_sharp, F, L, K}.
 * `out` must hold 8*B int32 (host). Synchronises. */
int32_t llsr_batch_counts(llsr_handle* h, int32_t* out);

/* Per-kernel device time (ms per batch, averaged over every batch enqueued since profiling was
 * enabled) from HIP events recorded on each batch's launch stream between its kernels, in the
 * order of llsr_kernel_name(k). Synchronises. Returns the number of kernels written (<= cap). */
int32_t llsr_kernel_times_ms(llsr_handle* h, float* out, int32_t cap);
const char* llsr_kernel_name(int32_t k);
/* Enable/disable per-kernel event timing; (re)enabling clears the accumulated averages. */
int32_t llsr_set_profiling(llsr_handle* h, int32_t enable);

/* ---- FeatureAssociation scan-to-scan LM (updateTransformation, featureAssociation.cpp:2505-2535) ----
 * Two-step LM between consecutive scans: surf phase (rx, rz, ty; FA:1699-2010) then corner
 * phase (ry, tx, tz; FA:1580-1697, 2013-2143), each <= 100 iterations, kNN-1 + ring-constrained
 * neighbour search every 5th iteration. Inputs per scan (float4 x, y, z, intensity, LOAM frame):
 * cornerPointsSharp and surfPointsFlat (with the 160 shadow points, FA:1310-1314) of the
 * current scan; laserCloudCornerLast / laserCloudSurfLast of the previous one (after
 * TransformToEnd + shadow points, FA:2660-2712). */
typedef struct llsr_s2s_report {
  int32_t surf_iterations;    /* iterCount1 when the surf loop ended (index of the converged step, or 100) */
  int32_t corner_iterations;  /* iterCount2 likewise (the reference's odometry_itertimes, FA:2800) */
  int32_t n_surf_corr;        /* correspondences at the last evaluated iteration of each phase */
  int32_t n_corner_corr;
  int32_t degenerate;         /* isDegenerate after the call (member state, FA:1975-1980) */
  int32_t skipped;            /* 1: last clouds too small, transformCur untouched (FA:2506) */
  float transform_cur[6];     /* rx, ry, rz, tx, ty, tz after updateTransformation */
  float ms;
} llsr_s2s_report;

/* The 160 virtual shadow points of GenerateShadowPoint (FA:412-439), float4 [160]. */
int32_t llsr_shadow_points(float* out_xyzi);

typedef struct llsr_s2s_batch {
  int32_t n_problems;
  const float* sharp;       const int64_t* sharp_off;        /* cornerPointsSharp */
  const float* flat;        const int64_t* flat_off;         /* surfPointsFlat + shadow points */
  const float* corner_last; const int64_t* corner_last_off;  /* laserCloudCornerLast */
  const float* surf_last;   const int64_t* surf_last_off;    /* laserCloudSurfLast */
  float* transform_cur;     /* [P][6] in/out */
  int32_t* is_degenerate;   /* [P] in/out (member state) */
  llsr_s2s_report* report;  /* [P] out (device memory) */
} llsr_s2s_batch;

/* Size the scan-to-scan buffers (problems per batch, points per cloud). */
int32_t llsr_scan2scan_reserve(llsr_handle* h, int32_t max_problems, int32_t max_sharp, int32_t max_flat,
                               int32_t max_corner_last, int32_t max_surf_last);
/* Enqueue a batch on `hip_stream` (NULL: the handle's own non-blocking stream); fully asynchronous: every
 * iteration runs inside one kernel. LLSR_ERANGE is reported by a later call's check of the
 * device error flag (llsr_scan2scan_check) when a cloud exceeded the reservation. */
int32_t llsr_scan2scan_batch(llsr_handle* h, const llsr_s2s_batch* batch, void* hip_stream);
/* Synchronise the last scan-to-scan batch and report capacity violations (LLSR_ERANGE). */
int32_t llsr_scan2scan_check(llsr_handle* h);
/* One scan from host buffers; reserves as needed; transform_cur / is_degenerate in/out. */
int32_t llsr_scan2scan(llsr_handle* h, const float* sharp, int32_t n_sharp, const float* flat, int32_t n_flat,
                       const float* corner_last, int32_t n_corner_last, const float* surf_last,
                       int32_t n_surf_last, float* transform_cur, int32_t* is_degenerate,
                       llsr_s2s_report* rep);


/* ---- MapOptimization scan-to-map (scan2MapOptimization, mapOptmization.cpp:1572-1610) ----
 * A batch of independent problems, one per scan: the scan's corner queries
 * (laserCloudCornerScanDS, MO:1244-1247) and surf queries (laserCloudSurfTotalLastDS,
 * MO:1259-1266), the corner / surf local maps (laserCloud{Corner,Surf}FromMapDS, MO:1225-1231)
 * and transformTobeMapped. Clouds are float4 rows (x, y, z, intensity) concatenated over the
 * batch with int64 offsets [P+1], all device-resident. The handle's config supplies
 * iterCountThres, step_size, stop_thres and mode (LLSR_MODE_FAITHFUL keeps the reference's
 * commented-out pose update, MO:1539-1545; LLSR_MODE_LM_APPLIED applies it). */
typedef struct llsr_s2m_batch {
  int32_t n_problems;
  const float* corner_q;   const int64_t* corner_q_off;
  const float* surf_q;     const int64_t* surf_q_off;
  const float* corner_map; const int64_t* corner_map_off;
  const float* surf_map;   const int64_t* surf_map_off;
  float* pose;               /* [P][6] in/out: roll, pitch, yaw, x, y, z (LOAM frame) */
  llsr_lm_report* report;    /* [P] out (device memory); report.ms is 0 in batch mode */
} llsr_s2m_batch;

/* Size the scan-to-map buffers: up to `max_problems` problems per batch with at most the given
 * points per cloud. Replaces MO's per-scan kd-tree allocation (MO:1575-1576). */
int32_t llsr_scan2map_reserve(llsr_handle* h, int32_t max_problems, int32_t max_corner_map,
                              int32_t max_surf_map, int32_t max_corner_q, int32_t max_surf_q);
/* Run the batch on `hip_stream` (NULL: the handle's own non-blocking stream). The LM's iteration count is data
 * dependent, so the call waits on the stream every few iterations to stop once every problem
 * has converged or reached iterCountThres; it returns when the batch is complete.
 * LLSR_ERANGE: a cloud exceeds the reserved capacity (nothing written for that problem). */
int32_t llsr_scan2map_batch(llsr_handle* h, const llsr_s2m_batch* batch, void* hip_stream);
/* Device time of the scan-to-map batches run since profiling was (re)enabled
 * (llsr_set_profiling), from HIP events on the launch stream. */
typedef struct llsr_s2m_stats {
  int32_t batches;
  int32_t iteration_launches;  /* k_s2m_iter launches, summed over batches */
  float grid_ms;               /* setup + cell-table build, summed */
  float iterate_ms;            /* first to last LM launch incl. the host's convergence polls, summed */
} llsr_s2m_stats;
int32_t llsr_scan2map_stats(llsr_handle* h, llsr_s2m_stats* out);
/* Device time of the scan-to-scan batches (llsr_scan2scan_batch, and the LM inside
 * llsr_odometry_batch) run since profiling was (re)enabled, from HIP events on the launch stream.
 * Profiling syncs the stream after each batch. */
typedef struct llsr_s2s_stats {
  int32_t batches;
  int32_t reserved;
  float grid_ms; /* cell grids of the last clouds (kd-tree build, FA:2313-2314), summed */
  float lm_ms;   /* k_s2s_lm: both LM phases of every problem (FA:2505-2535), summed */
} llsr_s2s_stats;
int32_t llsr_scan2scan_stats(llsr_handle* h, llsr_s2s_stats* out);
/* ---- Split-correspondence scan-to-map for multi-GPU (BASELINE.json configs[4]) ----
 * The optimisation of llsr_scan2map_batch driven one LM iteration at a time, so that the
 * per-problem normal equations can be summed across GPUs between the Jacobian build and the
 * solve. Rank r of W evaluates only its share of every problem's queries (256-query blocks b of
 * each kind with b % W == r) and writes int64 fixed-point partial sums, LLSR_NE_WORDS per
 * problem: AtA upper triangle (21, row-major), AtB (6), sum |coeff.intensity|, #corner, #surf
 * correspondences, 2 spare; every term is rounded once to a multiple of 2^-30 before it is
 * added. Range: a term must satisfy |v| < 2^32 and the sums stay exact while sum |term| < 2^33 per
 * word (e.g. 20k correspondences with |J|^2 up to 4e5, points ~600 m away); a non-finite or
 * out-of-range term contributes 0, is counted, and the step returns LLSR_ERANGE. Integer sums are associative, so the summed words, and therefore every pose, are
 * bit-identical for any W and any all-reduce order (they differ from llsr_scan2map_batch's float
 * sums only by that rounding: well inside the 1e-4 pose tolerance). Per batch:
 *   llsr_scan2map_shard_begin(h, batch, stream)              (reserve as for llsr_scan2map_batch)
 *   up to iterCountThres times:
 *     llsr_scan2map_shard_partial(h, r, W, d_ne, stream)     d_ne: int64 [P][LLSR_NE_WORDS], device
 *     the caller sums d_ne over the W ranks in place (e.g. an RCCL all-reduce on `stream`)
 *     llsr_scan2map_shard_step(h, d_ne, &n_active, stream)   n_active NULL: no host sync
 *     stop once n_active == 0 (every rank sees the same count: no extra collective)
 *   llsr_scan2map_shard_end(h, stream)                        pose + report into the batch arrays
 * A handle holds one scan-to-map batch at a time (llsr_scan2map_batch / llsr_scan2map close an
 * open shard batch). */
#define LLSR_NE_WORDS 32
int32_t llsr_scan2map_shard_begin(llsr_handle* h, const llsr_s2m_batch* batch, void* hip_stream);
int32_t llsr_scan2map_shard_partial(llsr_handle* h, int32_t rank, int32_t world, int64_t* d_ne, void* hip_stream);
int32_t llsr_scan2map_shard_step(llsr_handle* h, const int64_t* d_ne, int32_t* n_active, void* hip_stream);
int32_t llsr_scan2map_shard_end(llsr_handle* h, void* hip_stream);

/* One problem from host buffers (the reference's call shape: scan2MapOptimization on the
 * member clouds); reserves as needed; `pose` in/out; rep->ms = device time. */
int32_t llsr_scan2map(llsr_handle* h, const float* corner_q, int32_t n_corner_q, const float* surf_q,
                      int32_t n_surf_q, const float* corner_map, int32_t n_corner_map,
                      const float* surf_map, int32_t n_surf_map, float* pose, llsr_lm_report* rep);


/* ---- End-to-end odometry (runFeatureAssociation, featureAssociation.cpp:2742-2853) ----
 * B independent sequences (slots). Each call consumes one device-resident scan per slot (as
 * llsr_process_batch) and runs, without leaving the device: the ImageProjection + feature stage,
 * then updateTransformation against the slot's last clouds (FA:2505-2535), integrateTransformation
 * (FA:2537-2568, transformSum) and publishCloudsLast (FA:2660-2717): TransformToEnd of the
 * less-sharp / less-flat clouds, which become the slot's last clouds (+ the 160 shadow points on
 * the surf side), and of the sharp / flat clouds (MapOptimization's scan inputs). A slot's first
 * scan runs checkSystemInitialization (FA:2291-2315) instead. transformCur carries over to the
 * next scan as the LM's initial guess. Requires LLSR_MODE_LM_APPLIED (LLSR_ENOSYS otherwise): in
 * the faithful mode updateInitialGuess (FA:2790) overwrites transformCur from the /odom2 topic,
 * which has no input here. One host sync per call (the feature counts size the packed clouds). */
typedef struct llsr_odom_slot {
  int32_t frames;            /* scans this slot has consumed */
  int32_t n_corner_last;     /* laserCloudCornerLastNum after the last scan */
  int32_t n_surf_last;       /* laserCloudSurfLastNum (incl. the 160 shadow points) */
  int32_t n_corner_scan;     /* laserCloudCornerScan = TransformToEnd(cornerPointsSharp); 0 on frame 1 */
  int32_t n_surf_scan;       /* laserCloudSurfScan = TransformToEnd(surfPointsFlat + shadow); 0 on frame 1 */
  float transform_cur[6];    /* transformCur after updateTransformation */
  float transform_sum[6];    /* transformSum after integrateTransformation */
  llsr_s2s_report lm;        /* the last scan's updateTransformation (skipped = 1 on frame 1) */
} llsr_odom_slot;
int32_t llsr_odometry_batch(llsr_handle* h, const float* d_xyzi, const int64_t* d_offsets, int32_t B,
                            void* hip_stream);
/* Slot b's state after the last call; the float4 cloud buffers (host, may be NULL) receive the
 * last clouds and the scan clouds (capacity H*W + 160 points each). Synchronises. */
int32_t llsr_odometry_fetch(llsr_handle* h, int32_t b, llsr_odom_slot* out, float* corner_last, float* surf_last,
                            float* corner_scan, float* surf_scan);
/* Start every slot over: transformCur / transformSum = 0, no last clouds, FA carry-over reset. */
int32_t llsr_odometry_reset(llsr_handle* h);

/* ---- MapOptimization local map (llsr_map.hip) ----
 * The keyframe store of saveKeyFramesAndFactor (MO:1686-1752) kept in HBM, the local-map assembly
 * of extractSurroundingKeyFrames (MO:1096-1231, both branches: the key-pose radius search of the
 * VLP-16 block, enable_loop_closure false at CFG:23, and the recent-keyframe queue of the VLP-32c /
 * HDL-64E blocks, enable_loop_closure true at CFG:91, 159) and the downSizeFilter* VoxelGrids
 * (MO:92-104; downsampleCurrentScan MO:1234-1267), on the device. A llsr_map is independent of any
 * llsr_handle, one per mapped sequence; it owns a non-blocking stream used when hip_stream is NULL.
 * Point clouds are float4 x, y, z, intensity. VoxelGrid = pcl::VoxelGrid<PointXYZI>::filter
 * (downsample_all_data, 0 min points): same voxel set and output order (ascending voxel index) as
 * PCL, each centroid summed in the order libstdc++'s std::sort leaves PCL's index_vector. */
typedef struct llsr_map llsr_map;
typedef struct llsr_map_config {
  float surrounding_radius;  /* surrounding_keyframe_search_radius, 50 m (CFG:26) */
  float keypose_leaf;        /* downSizeFilterSurroundingKeyPoses, 1.0 (MO:99) */
  float corner_leaf;         /* downSizeFilterCorner, 0.2 (MO:92) */
  float surf_leaf;           /* downSizeFilterSurf, 0.4 (MO:93) */
  float outlier_leaf;        /* downSizeFilterOutlier, 0.4 (MO:94) */
  /* mapping.enable_loop_closure (CFG:23 / 91 / 159). Non-zero selects the branch of
   * extractSurroundingKeyFrames at MO:1099-1151: the local map is the last
   * surrounding_keyframe_search_num keyframes, refilled from the newest backwards while the queue
   * is short, then one pop-oldest / push-newest per call whenever the newest keyframe index changed
   * (latestFrameID, MO:1126-1134). The loop-closure ICP thread itself is commented out in the
   * reference (MO:174), so this flag changes only the local map. */
  int32_t enable_loop_closure;
  int32_t surrounding_keyframe_search_num;  /* 50 (CFG:27 / 95 / 163) */
} llsr_map_config;
/* VLP-16 block: radius branch (enable_loop_closure 0), search num 50, the leaves above. */
int32_t llsr_map_config_default(llsr_map_config* cfg);
/* The block of loam_config.yaml for `lidar` (LLSR_LIDAR_VLP16: CFG:20-27; LLSR_LIDAR_HDL64E:
 * CFG:156-163, enable_loop_closure 1). */
int32_t llsr_map_config_lidar(llsr_map_config* cfg, int32_t lidar);
llsr_map* llsr_map_create(const llsr_map_config* cfg, int32_t hip_device);
void llsr_map_destroy(llsr_map* m);
const char* llsr_map_last_error(const llsr_map* m);
/* Drop every keyframe and the surrounding-keyframe list. */
int32_t llsr_map_reset(llsr_map* m);
/* VoxelGrid of S independent clouds packed in d_in (device float4); off[S+1] and leaf[S] are host
 * arrays; d_out (device, capacity off[S] points) receives the S results packed, out_off[S+1]
 * (host) their offsets. Synchronises hip_stream. */
int32_t llsr_map_voxel_grid(llsr_map* m, const float* d_in, const int64_t* off, int32_t S, const float* leaf,
                            float* d_out, int64_t* out_off, void* hip_stream);
/* downsampleCurrentScan (MO:1234-1267). Inputs (device float4): laserCloudCornerLast, SurfLast,
 * OutlierLast, CornerScan, SurfScan. d_out (capacity n_cl + n_sl + n_ol + n_cs + n_ss + n_sl +
 * n_ol points) receives, packed in this order: CornerLastDS (corner leaf), SurfLastDS (surf leaf),
 * OutlierLastDS (outlier leaf), CornerScanDS, SurfScanDS, SurfTotalLastDS (= surf leaf over
 * SurfLastDS + OutlierLastDS); out_off[7] (host) their offsets. Synchronises. */
int32_t llsr_map_downsample_scan(llsr_map* m, const float* corner_last, int32_t n_cl, const float* surf_last,
                                 int32_t n_sl, const float* outlier_last, int32_t n_ol, const float* corner_scan,
                                 int32_t n_cs, const float* surf_scan, int32_t n_ss, float* d_out, int64_t* out_off,
                                 void* hip_stream);
/* saveKeyFramesAndFactor's store (MO:1686-1752): key pose x, y, z, roll, pitch, yaw (PointTypePose;
 * cloudKeyPoses3D = x, y, z with intensity = the returned keyframe index) and the keyframe's corner
 * (laserCloudCornerScan), surf (SurfLastDS) and outlier (OutlierLastDS) clouds, copied into the
 * store (device or host pointers). Returns the index (>= 0) or an error. */
int32_t llsr_map_add_keyframe(llsr_map* m, const float pose[6], const float* corner, int32_t n_corner,
                              const float* surf, int32_t n_surf, const float* outlier, int32_t n_outlier,
                              void* hip_stream);
int32_t llsr_map_num_keyframes(const llsr_map* m);
typedef struct llsr_map_report {
  int32_t n_in_radius;     /* key poses within surrounding_radius (MO:1157-1164); 0 with loop closure */
  int32_t n_poses_ds;      /* surroundingKeyPosesDS size (MO:1166-1167); 0 with loop closure */
  int32_t n_keyframes;     /* surroundingExistingKeyPosesID size after the update (loop closure:
                              recentCornerCloudKeyFrames size) */
  int32_t n_transformed;   /* keyframes newly added to the list this call (MO:1205-1220; loop
                              closure: pushed onto the queue, MO:1115-1120 / 1138-1143) */
  int64_t n_corner_map;    /* laserCloudCornerFromMap before / after VoxelGrid */
  int64_t n_surf_map;      /* laserCloudSurfFromMap (surf + outlier keyframe clouds) */
  int64_t n_corner_ds;
  int64_t n_surf_ds;
  float ms;                /* wall time of the call */
} llsr_map_report;
/* extractSurroundingKeyFrames (MO:1096-1232) around robot_pos (currentRobotPosPoint = x, y, z of
 * transformAftMapped; unused with loop closure): the corner / surf local maps (…FromMapDS) into
 * d_corner / d_surf (device, capacities in points; LLSR_ERANGE with the sizes in rep when they do
 * not fit). Synchronises. */
int32_t llsr_map_extract(llsr_map* m, const float robot_pos[3], float* d_corner, int64_t cap_corner, float* d_surf,
                         int64_t cap_surf, llsr_map_report* rep, void* hip_stream);
/* surroundingExistingKeyPosesID (loop closure: the queue's keyframe indices, oldest first) after the
 * last extract; returns its length. */
int32_t llsr_map_keyframe_ids(const llsr_map* m, int32_t* out, int32_t cap);

/* ---- Mapping chain: ImageProjection -> FeatureAssociation -> MapOptimization::run ----
 * (mapOptmization.cpp:1854-1896.) Each llsr_mapping_batch call runs llsr_odometry_batch on the B
 * slots and then, for every slot that sends an AssociationOut this frame — FA counts the frames
 * after the first (the first scan sends nothing, FA:2781-2784) and sends on every
 * mapping_frequency_divider-th of them (FA:2818-2821; llsr_config.mapping_frequency_divider, 1 in
 * every config block; a value < 1 never sends, as in the reference) — OdometryToTransform of the published odometry
 * (tf2 round trip, FA:2612-2625 / utility.h:99-113), transformAssociateToMap (MO:458-581),
 * extractSurroundingKeyFrames on the slot's keyframe store (MO:1096-1232), downsampleCurrentScan
 * of the AssociationOut clouds (corner / surf last, the adjustOutlierCloud'ed IP outliers
 * FA:2600-2610, corner / surf scan; MO:1234-1267), scan2MapOptimization (MO:1572-1610: all slots
 * in one device batch, isDegenerate / matP carried per slot), transformUpdate (MO:583-589) and
 * saveKeyFramesAndFactor (MO:1612-1755; every frame is a keyframe there, saveThisKeyFrame is forced
 * true at MO:1629; the prior / between factors with the initial values as measurements leave
 * iSAM2's estimate at the initial values, so the key pose is transformTobeMapped for the first
 * keyframe and transformAftMapped after). Requires the handle's mode LLSR_MODE_LM_APPLIED
 * (the odometry's); `mo_mode` selects MapOptimization's own LM mode (LLSR_MODE_FAITHFUL: the pose
 * update at MO:1539-1545 stays commented out, as in the reference). map_cfg NULL selects the
 * config block of the handle's lidar (llsr_map_config_lidar: HDL-64E when num_vertical_scans is
 * 64, else VLP-16), which decides the local-map branch (enable_loop_closure). Synchronises per
 * call. An error from the MapOptimization part of a call (after the odometry advanced) leaves every
 * slot's MapOptimization members (poses, keyframes, local-map queue, LM members) as before the call. */
typedef struct llsr_mapping_slot {
  int32_t frames;               /* scans consumed by the slot (odometry frames) */
  int32_t mo_frames;            /* MapOptimization::run iterations = frames - 1 once frames >= 2 */
  int32_t keyframes;            /* cloudKeyPoses3D size */
  int32_t lm_ran;               /* the last frame's map passed MO:1573 (corner > 10, surf > 100) */
  float transform_sum[6];       /* OdometryToTransform of the last published odometry */
  float transform_tobe_mapped[6];
  float transform_bef_mapped[6];
  float transform_aft_mapped[6];
  int32_t n_corner_q;           /* laserCloudCornerScanDSNum (the corner queries) */
  int32_t n_surf_q;             /* laserCloudSurfTotalLastDSNum (the surf queries) */
  llsr_lm_report lm;            /* the last frame's scan2MapOptimization (iterations 0 when skipped) */
  llsr_map_report map;          /* the last frame's extractSurroundingKeyFrames */
} llsr_mapping_slot;
/* Allocate the per-slot MapOptimization state (max_batch slots, map_cfg NULL = the reference's
 * leaves and radius) and start every slot over (also resets the odometry). */
int32_t llsr_mapping_init(llsr_handle* h, int32_t mo_mode, const llsr_map_config* map_cfg);
int32_t llsr_mapping_batch(llsr_handle* h, const float* d_xyzi, const int64_t* d_offsets, int32_t B,
                           void* hip_stream);
int32_t llsr_mapping_fetch(llsr_handle* h, int32_t b, llsr_mapping_slot* out);
/* cloudKeyPoses6D of slot b: x, y, z, roll, pitch, yaw per keyframe into out[6*cap]; returns the
 * keyframe count (may exceed cap). */
int32_t llsr_mapping_keyposes(llsr_handle* h, int32_t b, float* out, int32_t cap);
/* Start every slot over: odometry, poses, keyframe stores. */
int32_t llsr_mapping_reset(llsr_handle* h);
/* Host-only (no device): the pose glue llsr_mapping_batch applies per frame — OdometryToTransform
 * of FA's transformSum (tf2 round trip) into transform_sum, then transformAssociateToMap with the
 * given transformBefMapped / transformAftMapped into transform_tobe_mapped (and transform_incre,
 * may be NULL). */
int32_t llsr_mapping_associate(const float transform_sum_fa[6], const float transform_bef_mapped[6],
                               const float transform_aft_mapped[6], float transform_sum[6],
                               float transform_tobe_mapped[6], float transform_incre[6]);


/* ---- FA end of scan on the FA node's thread (host side, no handle) ----
 * For a node whose FeatureAssociation thread owns its own clouds and calls llsr_scan2scan on its
 * own handle: integrateTransformation (FA:2537-2568, no IMU) updates
 * transform_sum in place from transformCur; TransformToEnd (FA:1414-1490, the
 * use_imu_undistortion == false branch) moves n float4 rows (x, y, z, intensity; intensity =
 * ring + relTime / 10 as adjustDistortion leaves it) to the scan's end with transformCur, as
 * publishCloudsLast does for the less-sharp / less-flat and sharp / flat clouds (FA:2666-2707).
 * out_xyzi may equal in_xyzi. Bit-identical to the device odometry path (llsr_odometry_batch). */
int32_t llsr_integrate_transformation(float transform_sum[6], const float transform_cur[6]);
int32_t llsr_transform_to_end(const float transform_cur[6], const float* in_xyzi, int32_t n, float* out_xyzi);

/* ---- TransformFusion (transformFusion.cpp) ----
 * The fourth node of the reference fuses the 10 Hz scan-to-scan odometry with the slower mapped
 * pose. It is scalar host work per message, so these entry points run on the host side of the
 * library (no device, no handle), with the reference's float / double typing: tf2's
 * Quaternion::setRPY / Matrix3x3::getRPY in double, transformAssociateToMap on floats (the same
 * routine as MO:458-581, TF:65-186). The odometry messages carry the nav_msgs/Odometry fields the
 * nodes read and write. */
typedef struct llsr_odometry_msg {
  double orientation[4];    /* pose.pose.orientation x, y, z, w */
  double position[3];       /* pose.pose.position */
  double twist_angular[3];  /* twist.twist.angular (MO's transformBefMapped[0..2]) */
  double twist_linear[3];   /* twist.twist.linear (MO's transformBefMapped[3..5]) */
} llsr_odometry_msg;
typedef struct llsr_fusion_state {  /* TransformFusion's members (transformFusion.h) */
  float transform_sum[6];
  float transform_incre[6];
  float transform_mapped[6];
  float transform_bef_mapped[6];
  float transform_aft_mapped[6];
} llsr_fusion_state;
/* The constructor's zeros (TF:51-57). */
int32_t llsr_fusion_init(llsr_fusion_state* st);
/* How the publishers encode a pose: orientation = (-q.y, -q.z, q.x, q.w) of
 * setRPY(pose[2], -pose[0], -pose[1]), position = pose[3..5]; twist = twist6 (NULL: zeros).
 * FeatureAssociation::publishOdometry (FA:2612-2625: transformSum, no twist),
 * MapOptimization::publishTF (MO:704-723: transformAftMapped, twist = transformBefMapped),
 * TransformFusion's /integrated_to_init (TF:193-206: transformMapped, no twist). */
int32_t llsr_pose_to_odometry(const float pose[6], const float twist6[6], llsr_odometry_msg* out);
/* OdometryToTransform (UT:99-113): getRPY of Quaternion(o.z, -o.x, -o.y, o.w) -> (-pitch, -yaw,
 * roll), position. */
int32_t llsr_odometry_to_transform(const llsr_odometry_msg* in, float transform[6]);
/* TransformFusion::laserOdometryHandler (TF:188-280): transform_sum from /laser_odom_to_init,
 * transformAssociateToMap, and the /integrated_to_init message (also the camera_init -> camera tf,
 * same rotation and translation). */
int32_t llsr_fusion_laser_odometry(llsr_fusion_state* st, const llsr_odometry_msg* laser_odometry,
                                   llsr_odometry_msg* integrated);
/* TransformFusion::odomAftMappedHandler (TF:282-304): transform_aft_mapped from the pose (getRPY
 * of Quaternion(o.z, -o.x, -o.y, o.w) -> -pitch, -yaw, roll), transform_bef_mapped from the twist. */
int32_t llsr_fusion_aft_mapped(llsr_fusion_state* st, const llsr_odometry_msg* odom_aft_mapped);

/* ---- Input wire formats (llsr_input.hip) ----
 * sensor_msgs/PointCloud2 (PointField datatype codes, sensor_msgs/msg/PointField.msg) decoded as
 * pcl::fromROSMsg<PointXYZI> (IP:196): x, y, z, intensity are taken from the fields of that name
 * whose datatype is FLOAT32 and count 1; any other field is ignored and an unmatched PointXYZI
 * field reads 0 (its default). Byte order is taken as-is (PCL ignores is_bigendian). */
#define LLSR_PC2_FLOAT32 7
#define LLSR_PC2_MAX_FIELDS 16
typedef struct llsr_pc2_field {
  char name[16];
  int32_t offset;    /* byte offset in the point */
  int32_t datatype;  /* PointField.datatype */
  int32_t count;
} llsr_pc2_field;
typedef struct llsr_pc2_layout {  /* the message's fields + point_step (constant per sensor) */
  int32_t point_step;
  int32_t num_fields;
  llsr_pc2_field fields[LLSR_PC2_MAX_FIELDS];
} llsr_pc2_layout;
typedef struct llsr_pc2_msg {     /* one message of the batch */
  int64_t data_offset;            /* first byte of its `data` in the packed device buffer */
  int32_t width, height;          /* points = width * height */
  int32_t row_step;               /* bytes per row (organized clouds, height > 1) */
  int32_t pad;
} llsr_pc2_msg;
/* Decode B messages whose data bytes are packed in d_data (device) into float4 x, y, z, intensity
 * points packed in d_out (device, capacity sum(width * height)), in row-major point order; writes
 * the point offsets to out_off[B+1] (host) and, if not NULL, to d_out_off[B+1] (device) — the
 * inputs llsr_process_batch / llsr_odometry_batch take. NaN points are kept (those calls remove
 * them, IP:198). Synchronises hip_stream. */
int32_t llsr_decode_pointcloud2(const llsr_pc2_layout* layout, const uint8_t* d_data, const llsr_pc2_msg* msgs,
                                int32_t B, float* d_out, int64_t* out_off, int64_t* d_out_off, void* hip_stream);
/* KITTI velodyne sequences (offlineKittiService IP:224-248, KittiLoader imageProjection.h:127-200):
 * a frame file holds float32 x, y, z, reflectance records; like the reference, at most
 * LLSR_KITTI_MAX_FLOATS floats are read and floor(floats / 4) points kept. */
#define LLSR_KITTI_MAX_FLOATS 1000000
/* Number of consecutive frames <dir>/%06d.bin starting at 0. */
int32_t llsr_kitti_count(const char* velodyne_dir);
/* One frame into a host buffer (capacity cap points); *n = points (LLSR_ERANGE if > cap). */
int32_t llsr_kitti_read(const char* path, float* xyzi, int32_t cap, int32_t* n);
/* Frames first .. first+B-1 of <dir> into d_xyzi (device, capacity cap_points) with one pinned
 * upload; point offsets to off[B+1] (host) and, if not NULL, d_off[B+1] (device). Synchronises. */
int32_t llsr_kitti_load(const char* velodyne_dir, int32_t first, int32_t B, float* d_xyzi, int64_t cap_points,
                        int64_t* off, int64_t* d_off, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* LLSR_H_ */
