/*
 * pn2hip.h — C ABI of the MI355X (gfx950) PointNet++ geometric hot path.
 *
 * This is the drop-in boundary. Each entry point replaces one TensorFlow custom op (or one
 * inline TF graph fragment) of the reference and keeps its argument meaning:
 *
 *   reference op / fragment                                     → entry point here
 *   FarthestPointSample  tf_sampling.cpp:94-123, .cu:105-170     → pn2_fps (+_gather, _chain)
 *   GatherPoint          tf_sampling.cpp:125-148, .cu:172-181    → pn2_gather_point
 *   GatherPointGrad      tf_sampling.cpp:150-178, .cu:183-192    → pn2_gather_point_grad
 *   ProbSample           tf_sampling.cpp:66-92, .cu:7-104,197-201 → pn2_prob_sample
 *   QueryBallPoint       tf_grouping.cpp:66-106, _g.cu:3-36      → pn2_ball_query,
 *                                                                  pn2_ball_query_grid
 *   SelectionSort        tf_grouping.cpp:108-137, _g.cu:83-123   → pn2_select_top_k
 *   knn_point            tf_grouping.py:48-73                    → pn2_knn_point
 *   GroupPoint           tf_grouping.cpp:139-171, _g.cu:40-57    → pn2_group_point
 *   GroupPointGrad       tf_grouping.cpp:174-208, _g.cu:61-78    → pn2_group_point_grad
 *   ThreeNN              tf_interpolate.cpp:157-187, :60-103     → pn2_three_nn,
 *                                                                  pn2_three_nn_grid,
 *                                                                  pn2cpu_three_nn (host)
 *   ThreeInterpolate     tf_interpolate.cpp:191-222, :107-127    → pn2_three_interpolate,
 *                                                                  pn2cpu_three_interpolate
 *   ThreeInterpolateGrad tf_interpolate.cpp:225-262, :131-153    → pn2_three_interpolate_grad,
 *                                                                  pn2cpu_three_interpolate_grad
 *   IDW weights          pointnet_util.py:219-222                → pn2_idw_weights
 *   sample_and_group     pointnet_util.py:16-58 (SSG), :180-191  → pn2_sample_and_group,
 *                                                                  pn2_group_concat
 *   pointnet_fp_module   pointnet_util.py:218-226 (geometry)     → pn2_fp_fused,
 *                                                                  pn2_fp_grid_fused,
 *                                                                  pn2_fp_apply
 *   AttentionLayer.call  attention_layer.py:29-45 (reduction)    → pn2_attn_reduce,
 *                                                                  pn2_attn_reduce_grad
 *   SA pooling           pointnet_util.py:130-145, :200          → pn2_group_pool
 *   pointnet_sa_module   pointnet_util.py:106-145 (group, conv2d  → pn2_group_mlp
 *     MLP, pooling; tf_util.py:120-185 conv2d + batch_norm)
 *   pointnet_sa_module_attention(_and_pooling)                   → pn2_group_mlp_attention
 *                        attention_layer.py:229-338
 *   pointnet_fp_module   pointnet_util.py:218-238 (interp + MLP)  → pn2_fp_mlp
 *   conv1d head          tf_util.py:52-117, pointnet2_sem_seg.py  → pn2_shared_mlp
 *                        :57-60 (fc1, fc2)
 *   get_subset           scannet_dataset/data_transformation.py  → pn2_scene_bbox,
 *                        :70-154 (training crop sampler)           pn2_crop_sample
 *   whole-scene chunker  scannet_dataset/complete_scene_loader.py → pn2_subvolume_select,
 *                        :4-117 (subvolume selection, gathers)     pn2_gather_rows
 *
 * (reference paths are under pointnet2_tensorflow/tf_ops/{sampling,grouping,interpolation_3d},
 *  pointnet2_tensorflow/utils and attention_points/attention_scannet.)
 *
 * Conventions (all entry points):
 *  - every buffer is a caller-owned DEVICE pointer, row-major, channel-last, contiguous;
 *    float = IEEE fp32, indices int32 — the reference's tensor dtypes;
 *  - every launch goes on `stream` (a hipStream_t; NULL = legacy default stream); nothing
 *    synchronises, nothing allocates on the device (the first sampler call pins one 4-byte
 *    host word for device fault codes), so every call can be captured into a hipGraph;
 *  - return 0 on success, PN2_EINVAL (-22) for a shape/attribute error (where the reference
 *    raises InvalidArgument through OP_REQUIRES), PN2_EFAULT (-14) when an earlier sampler
 *    launch reported a device fault (pn2_fault_status), or a positive hipError_t from the
 *    launch.
 */
#ifndef PN2HIP_H
#define PN2HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* pn2_stream_t; /* hipStream_t */

#define PN2_OK 0
#define PN2_EINVAL (-22)
#define PN2_EFAULT (-14) /* an earlier launch stored a device fault code (pn2_fault_status)   */
#define PN2_ENOTSUP (-95) /* valid arguments this device / path does not take (see each call)  */

/* device fault codes (pn2_fault_status) */
#define PN2_FAULT_FPS_POLL 1 /* culled sampler: a cold wave waited past its poll bound for
                                 centres the hot wave never published; that launch's indices
                                 are not trustworthy                                      */

/* pn2_fps_gather_sched schedules (all give identical outputs) */
#define PN2_FPS_AUTO 0           /* the library's choice by N (what pn2_fps* run)            */
#define PN2_FPS_BLOCKSCAN 1      /* one block-wide argmax per pick (the v9 register sampler) */

/* flags of pn2_group_concat / pn2_sample_and_group */
#define PN2_USE_XYZ 1  /* concat the centred xyz with the grouped features (use_xyz=True)      */
#define PN2_XYZ_LAST 2 /* MSG order [points, xyz] (pointnet_util.py:191) instead of SSG
                          [xyz, points] (pointnet_util.py:52)                                 */

/* pn2_group_pool modes (pointnet_util.py:130-145) */
#define PN2_POOL_MAX 0
#define PN2_POOL_AVG 1
#define PN2_POOL_WEIGHTED_AVG 2
#define PN2_POOL_MAX_AND_AVG 3
#define PN2_POOL_NONE (-1) /* pn2_group_mlp: per-point output, no pooling */

/* shared-MLP layers (pn2_group_mlp / pn2_fp_mlp / pn2_shared_mlp) */
#define PN2_MLP_MAX_LAYERS 6
#define PN2_MLP_RELU 1 /* activation_fn = tf.nn.relu (tf_util.conv2d's default) */

typedef struct pn2_mlp_layer {
  const void* packed; /* pn2_mlp_pack output (device, 16-byte aligned)                    */
  int cin, cout;      /* the conv's input / output channels                              */
  int flags;          /* PN2_MLP_RELU                                                    */
} pn2_mlp_layer;

const char* pn2_version(void);
const char* pn2_strerror(int status);

/* Measurement utility (bench.py's copy peak; no operator uses it): copy `bytes` (a multiple
 * of 16, both pointers 16-byte aligned) with float4 loads and stores over 16 workgroups per
 * CU of `cus` CUs. */
int pn2_copy_f4(const void* src, void* dst, size_t bytes, int cus, pn2_stream_t stream);

/* ---------------------------------------------------------------- sampling -------------- */

/* Farthest-point sampling. xyz (B,N,3) → idx (B,npoint). idx[b,0]=0; each next index is the
 * argmax of the running min squared distance, ties broken exactly like the reference's
 * 512-thread block reduction: smallest (k mod 512), then smallest (k div 512)
 * (tf_sampling_g.cu:130-165). Distances are ((dx*dx+dy*dy)+dz*dz) in fp32 without FMA.
 * npoint must be > 0 (tf_sampling.cpp:99). N <= pn2_fps_max_points() needs no workspace;
 * larger N must use pn2_fps_ws. */
int pn2_fps(const float* xyz, int B, int N, int npoint, int32_t* idx, pn2_stream_t stream);
/* Same, also writing new_xyz (B,npoint,3) = gather_point(xyz, idx) (pointnet_util.py:34). */
int pn2_fps_gather(const float* xyz, int B, int N, int npoint, int32_t* idx, float* new_xyz,
                   pn2_stream_t stream);
int pn2_fps_max_points(void);
/* pn2_fps_gather with an explicit sampler schedule, per call (no process-wide state; used by
 * the parity tests and A/B timing). PN2_FPS_AUTO = pn2_fps_gather; the other schedules exist
 * only where the culled hot-set sampler is the default (4096 < N <= 16384) and return
 * PN2_EINVAL elsewhere. */
int pn2_fps_gather_sched(const float* xyz, int B, int N, int npoint, int32_t* idx,
                         float* new_xyz, int schedule, pn2_stream_t stream);
/* The device fault word: 0, or the PN2_FAULT_* code a sampler launch stored (valid once that
 * launch's stream has synchronised). clear != 0 resets it. The next pn2_fps* call also
 * reports a stored fault, as PN2_EFAULT, and resets it. */
int pn2_fault_status(int clear);
size_t pn2_fps_workspace_size(int B, int N);
int pn2_fps_ws(const float* xyz, int B, int N, int npoint, int32_t* idx, float* new_xyz,
               void* workspace, size_t workspace_bytes, pn2_stream_t stream);

/* The SSG sampler chain: stage 0 samples npoint[0] of the N points of each cloud, stage i
 * samples npoint[i] of stage i-1's output (pointnet2_sem_seg*.py:29-50 samples
 * 8192 -> 1024 -> 256 -> 64 -> 16). idx[i] (B,npoint[i]) and new_xyz[i] (B,npoint[i],3) are
 * exactly what pn2_fps_gather returns for that stage's input. N <= pn2_fps_max_points(),
 * npoint[i] <= 1024 for every stage that feeds another, 1 <= nstages <= 4. Host arrays of
 * device pointers. At most three launches on `stream`: a first stage over N > 1024 points as
 * the ordinary sampler; a check whether the remaining stages are prefixes of their input
 * (they are when that input is itself a sampler's output -- SA2 sampling SA1's picks -- and
 * no two points tie: csrc/fps.hip fps_prefix_holds; it leaves its verdict in the head of each
 * cloud's idx row of the first fused stage, which the next launch overwrites); then every
 * remaining stage fused in one launch (one workgroup per cloud: copies of the prefix, or a
 * stage of up to 1024 picks on the hot-set schedule, the same picks either way). */
int pn2_fps_chain(const float* xyz, int B, int N, int nstages, const int* npoint,
                  int32_t* const* idx, float* const* new_xyz, pn2_stream_t stream);
/* pn2_fps_chain plus the automatic-edge grid of stage 0's picks (the known points of the last
 * FP layer, pointnet2_sem_seg*.py:55 / pointnet_util.py:218): grid0 (pn2_grid_size(B,
 * npoint[0]) bytes, 16-byte aligned) gets exactly what pn2_grid_build(new_xyz[0], B,
 * npoint[0], 0, grid0) writes, up to the order of the points inside a cell. The culled
 * sampler builds it in its own workgroups after the last pick (npoint[0] <= 4096; otherwise
 * one pn2_grid_build launch follows on `stream`). new_xyz[0] must not be NULL. */
int pn2_fps_chain_grid(const float* xyz, int B, int N, int nstages, const int* npoint,
                       int32_t* const* idx, float* const* new_xyz, void* grid0,
                       size_t grid0_bytes, pn2_stream_t stream);
/* out (B,M,3) = inp[b, idx[b,j], :]; inp must have 3 channels (tf_sampling.cpp:131). */
int pn2_gather_point(const float* inp, const int32_t* idx, int B, int N, int M, float* out,
                     pn2_stream_t stream);
/* inp_g (B,N,3) = scatter-add of out_g (B,M,3) at idx; zero-fills inp_g first
 * (tf_sampling.cpp:174). Float atomics: summation order is not fixed. */
int pn2_gather_point_grad(const float* out_g, const int32_t* idx, int B, int N, int M,
                          float* inp_g, pn2_stream_t stream);
/* Categorical sampling (ProbSample). inp (B,N) weights, inpr (B,M) uniform draws in [0,1) →
 * out (B,M): per row, the first index whose inclusive prefix sum of inp reaches
 * inpr * (the row total), found by the reference's binary search (tf_sampling_g.cu:90-104).
 * The prefix sum repeats cumsumKernel's fp32 addition order (:7-88), so the indices equal
 * the reference's. workspace: pn2_prob_sample_workspace_size(B, N) bytes (the prefix sums,
 * tf_sampling.cpp:85-88). N = 0 with M > 0 is rejected (the reference reads cum[-1]). */
size_t pn2_prob_sample_workspace_size(int B, int N);
int pn2_prob_sample(const float* inp, const float* inpr, int B, int N, int M, float* workspace,
                    size_t workspace_bytes, int32_t* out, pn2_stream_t stream);

/* ---------------------------------------------------------------- grouping -------------- */

/* Ball query. For every query j: the first `nsample` points of xyz1 (in index order) with
 * max(sqrtf(d2),1e-20f) < radius; remaining slots repeat the first hit; pts_cnt = number
 * found (<= nsample) (tf_grouping_g.cu:3-36). A query with no hit gets idx 0 and pts_cnt 0
 * (the reference leaves that row uninitialised). radius > 0, nsample > 0
 * (tf_grouping.cpp:71,74). */
int pn2_ball_query(const float* xyz1, const float* xyz2, int B, int N, int M, float radius,
                   int nsample, int32_t* idx, int32_t* pts_cnt, pn2_stream_t stream);
/* The float T with  d2 < T  <=>  max(sqrtf(d2),1e-20f) < radius  for every fp32 d2 >= 0.
 * Host function (pure, no GPU). */
float pn2_ball_threshold(float radius);
/* ---- spatial grid (grid.h): the same results as the scans, faster on large clouds ----- *
 * pn2_grid_build: per cloud, bbox + counting sort of xyz (B,N,3) into cells of edge
 *   `cell_edge` (<= 0: ~2 points per cell of the bbox), grown until at most 32768 cells, into
 *   `grid` = caller-owned device memory of pn2_grid_size(B, N) bytes, 16-byte aligned.
 * pn2_ball_query_grid: pn2_ball_query over a grid built on xyz1 (cell_edge = radius is the
 *   fast choice; any radius > 0 is exact). N <= 131072.
 * pn2_three_nn_grid (interpolation section): three_nn over a grid built on the known points. */
size_t pn2_grid_size(int B, int N);
int pn2_grid_build(const float* xyz, int B, int N, float cell_edge, void* grid,
                   size_t grid_bytes, pn2_stream_t stream);
int pn2_ball_query_grid(const void* grid, const float* xyz2, int B, int N, int M, float radius,
                        int nsample, int32_t* idx, int32_t* pts_cnt, pn2_stream_t stream);
/* pn2_ball_query_grid plus the grouping of an xyz-only layer in the same kernel:
 * grouped_xyz (B,M,nsample,3) = xyz1[idx] - xyz2, i.e. pn2_group_concat with points = NULL
 * (pointnet_util.py:39-40, 55-56), bit for bit. xyz1 (B,N,3) is the cloud the grid was built
 * over. */
int pn2_ball_group_xyz_grid(const void* grid, const float* xyz1, const float* xyz2, int B, int N,
                            int M, float radius, int nsample, int32_t* idx, int32_t* pts_cnt,
                            float* grouped_xyz, pn2_stream_t stream);
/* pn2_ball_group_xyz_grid with features: ONE kernel for query_ball_point + group_point + the
 * centring and concat of sample_and_group (tf_grouping_g.cu:3-57, pointnet_util.py:38-52; MSG
 * order :186-191). new_points (B,M,nsample,3+C) = [xyz1[idx] - xyz2, points[idx]], or with
 * flags & PN2_XYZ_LAST [points[idx], xyz1[idx] - xyz2]; flags must hold PN2_USE_XYZ when C > 0
 * (C = 0: exactly pn2_ball_group_xyz_grid). idx / pts_cnt as pn2_ball_query_grid. Bit for bit
 * pn2_ball_query_grid followed by pn2_group_concat. */
int pn2_ball_group_grid(const void* grid, const float* xyz1, const float* points, int C,
                        int flags, const float* xyz2, int B, int N, int M, float radius,
                        int nsample, int32_t* idx, int32_t* pts_cnt, float* new_points,
                        pn2_stream_t stream);
/* pn2_ball_group_xyz_grid for nr radii (1 <= nr <= PN2_BQ_MAX_RADII) of the same queries in
 * ONE launch (MSG's SA1: pointnet_util.py:162-203, the radius loop): the cells of the largest
 * radius are walked once and every candidate is tested against each radius. Per radius r:
 * radii[r], nsample[r], idx[r] (B,M,nsample[r]), pts_cnt[r] (B,M), grouped_xyz[r]
 * (B,M,nsample[r],3) -- each exactly pn2_ball_group_xyz_grid's output for that radius. The
 * pointer arrays are host memory. The nr bitmasks per wave must fit 64 KB of LDS:
 * nr * ceil(N / 32) <= 4096 (PN2_EINVAL beyond: one launch per radius). */
#define PN2_BQ_MAX_RADII 3
int pn2_ball_group_xyz_grid_radii(const void* grid, const float* xyz1, const float* xyz2, int B,
                                  int N, int M, int nr, const float* radii, const int* nsample,
                                  int32_t* const* idx, int32_t* const* pts_cnt,
                                  float* const* grouped_xyz, pn2_stream_t stream);

/* ---- k nearest neighbours ---------------------------------------------------------- *
 * pn2_select_top_k: select_top_k / SelectionSort (tf_grouping.py:22-31, tf_grouping_g.cu:
 *   83-123): outi, out (B,m,n) = each row of dist (B,m,n) after the reference's k-step
 *   partial selection sort (first minimum by position, swapped to the front), i.e. the k
 *   smallest first, ties in the order those swaps leave them, the rest permuted by the same
 *   swaps. 0 < k <= min(n, 1024). workspace: pn2_select_top_k_workspace_size(B,m,k) bytes.
 * pn2_knn_point: knn_point (tf_grouping.py:48-73): val, idx (B,m,k) = the first k columns of
 *   select_top_k(k, dist) for dist[b,j,t] = sum over the c channels of (xyz1[b,t]-xyz2[b,j])^2
 *   (summed left to right); the (B,m,n) matrix is never materialised. */
int pn2_select_top_k(const float* dist, int B, int m, int n, int k, int32_t* outi, float* out,
                     int32_t* workspace, pn2_stream_t stream);
size_t pn2_select_top_k_workspace_size(int B, int m, int k);
int pn2_knn_point(const float* xyz1, const float* xyz2, int B, int n, int m, int c, int k,
                  float* val, int32_t* idx, pn2_stream_t stream);

/* out (B,M,nsample,C) = points[b, idx[b,j,k], :] (tf_grouping_g.cu:40-57). */
int pn2_group_point(const float* points, const int32_t* idx, int B, int N, int C, int M,
                    int nsample, float* out, pn2_stream_t stream);
/* grad_points (B,N,C) = scatter-add of grad_out (B,M,nsample,C); zero-fills first
 * (tf_grouping.cpp:204, tf_grouping_g.cu:61-78). Float atomics. */
int pn2_group_point_grad(const float* grad_out, const int32_t* idx, int B, int N, int C, int M,
                         int nsample, float* grad_points, pn2_stream_t stream);

/* Fused group + centre + concat (pointnet_util.py:39-56 SSG, :186-193 MSG):
 *   grouped_xyz (B,M,nsample,3) = xyz[idx] - new_xyz[j]            (optional, may be NULL)
 *   new_points  (B,M,nsample,Cout):
 *     points == NULL          → Cout = 3,      grouped_xyz
 *     !(flags & PN2_USE_XYZ)  → Cout = C,      points[idx]
 *     flags & PN2_XYZ_LAST    → Cout = C + 3,  [points[idx], grouped_xyz]   (MSG)
 *     otherwise               → Cout = 3 + C,  [grouped_xyz, points[idx]]   (SSG) */
int pn2_group_concat(const float* xyz, const float* points, const float* new_xyz,
                     const int32_t* idx, int B, int N, int C, int M, int nsample, int flags,
                     float* grouped_xyz, float* new_points, pn2_stream_t stream);
/* sample_and_group (pointnet_util.py:16-58, knn=False): FPS + gather + ball query + fused
 * group/centre/concat, four launches on `stream`. Outputs as in the reference:
 * fps_idx (B,npoint), new_xyz (B,npoint,3), idx (B,npoint,nsample), pts_cnt (B,npoint),
 * grouped_xyz (B,npoint,nsample,3) (may be NULL), new_points (B,npoint,nsample,Cout). */
int pn2_sample_and_group(const float* xyz, const float* points, int B, int N, int C,
                         int npoint, float radius, int nsample, int flags, int32_t* fps_idx,
                         float* new_xyz, int32_t* idx, int32_t* pts_cnt, float* grouped_xyz,
                         float* new_points, pn2_stream_t stream);

/* Several set-abstraction layers' ball query + fused group/centre/concat in ONE launch
 * (the SSG stack's SA2..SA4, or one MSG level's radii, which all wait for the same sampler).
 * Per layer the outputs equal pn2_ball_query (idx, pts_cnt) followed by pn2_group_concat
 * (new_points, grouped_xyz) with the same arguments, bit for bit. Limits: N <= 1024 points
 * per cloud (the cloud is staged in LDS), nsample <= 128, at most PN2_SA_MAX_LAYERS layers;
 * every layer has the same B. grouped_xyz may be NULL. */
#define PN2_SA_MAX_LAYERS 4
typedef struct pn2_sa_layer {
  const float* xyz;     /* (B,N,3) */
  const float* points;  /* (B,N,C) or NULL (then C is ignored and Cout = 3) */
  const float* new_xyz; /* (B,M,3) query centres */
  int N, C, M, nsample;
  float radius;
  int flags;            /* PN2_USE_XYZ | PN2_XYZ_LAST, as pn2_group_concat */
  int32_t* idx;         /* (B,M,nsample) */
  int32_t* pts_cnt;     /* (B,M) */
  float* grouped_xyz;   /* (B,M,nsample,3) or NULL */
  float* new_points;    /* (B,M,nsample,Cout) */
} pn2_sa_layer;
int pn2_ball_group_layers(const pn2_sa_layer* layers, int nlayers, int B, pn2_stream_t stream);

/* ---------------------------------------------------------------- interpolation --------- */

/* Three nearest known points (xyz2, (B,m,3)) of every unknown point (xyz1, (B,n,3)):
 * SQUARED distances ascending, ties keep the lower index, m<3 leaves idx 0 / dist +inf
 * (tf_interpolate.cpp:60-103). */
int pn2_three_nn(const float* xyz1, const float* xyz2, int B, int n, int m, float* dist,
                 int32_t* idx, pn2_stream_t stream);
/* out (B,n,C) = ((p[i1]*w1) + (p[i2]*w2)) + (p[i3]*w3)  (tf_interpolate.cpp:107-127). */
int pn2_three_interpolate(const float* points, const int32_t* idx, const float* weight, int B,
                          int m, int C, int n, float* out, pn2_stream_t stream);
/* grad_points (B,m,C) scatter-add (tf_interpolate.cpp:131-153); zero-fills first. */
int pn2_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight,
                               int B, int n, int C, int m, float* grad_points,
                               pn2_stream_t stream);
/* Host twins of the three ops the reference registers ONLY on DEVICE_CPU
 * (tf_interpolate.cpp:187,222,262): the same arguments minus the stream, HOST pointers,
 * synchronous (std::thread over clouds), the reference's fp32 arithmetic and order, so the
 * results equal threenn_cpu / threeinterpolate_cpu / threeinterpolate_grad_cpu bit for bit
 * (the grad's sums keep the reference's order within a cloud). */
int pn2cpu_three_nn(const float* xyz1, const float* xyz2, int B, int n, int m, float* dist,
                    int32_t* idx);
int pn2cpu_three_interpolate(const float* points, const int32_t* idx, const float* weight, int B,
                             int m, int C, int n, float* out);
int pn2cpu_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight,
                                  int B, int n, int C, int m, float* grad_points);
/* weight = (1/d)/sum(1/d), d = max(dist,1e-10)  (pointnet_util.py:219-222). */
int pn2_idw_weights(const float* dist, int B, int n, float* weight, pn2_stream_t stream);
/* pointnet_fp_module geometry (pointnet_util.py:218-226): three_nn + IDW weights +
 * three_interpolate + concat [interp (C2), points1 (C1)] → out (B,n,C2+C1).
 * points1 may be NULL (C1 must then be 0). */
int pn2_fp_fused(const float* xyz1, const float* xyz2, const float* points1, int C1,
                 const float* points2, int C2, int B, int n, int m, float* out,
                 pn2_stream_t stream);

/* Several pn2_fp_fused layers in ONE launch (the FP layers that wait for the same sampler):
 * per layer exactly pn2_fp_fused's output, bit for bit. At most PN2_FP_MAX_LAYERS layers,
 * every layer has the same B. */
#define PN2_FP_MAX_LAYERS 4
typedef struct pn2_fp_layer {
  const float* xyz1;    /* (B,n,3) unknown points */
  const float* xyz2;    /* (B,m,3) known points */
  const float* points1; /* (B,n,C1) or NULL (C1 = 0) */
  const float* points2; /* (B,m,C2) */
  int C1, C2, n, m;
  float* out;           /* (B,n,C2+C1) */
} pn2_fp_layer;
int pn2_fp_fused_layers(const pn2_fp_layer* layers, int nlayers, int B, pn2_stream_t stream);

/* three_nn over pn2_grid_build(xyz2 = the m known points): the same dist/idx as
 * pn2_three_nn. `unknown_grid` (optional, a grid over the n unknown points xyz1) only orders
 * the work so that neighbouring lanes share cells; with it xyz1 may be NULL. */
int pn2_three_nn_grid(const void* known_grid, const void* unknown_grid, const float* xyz1,
                      int B, int n, int m, float* dist, int32_t* idx, pn2_stream_t stream);
/* pn2_fp_fused from a previous three_nn: IDW weights of dist (B,n,3), interpolation of
 * points2 (B,m,C2) with idx (B,n,3), concat [interp, points1 (B,n,C1)]. `unknown_grid`
 * (optional, a grid over the n unknown points) only orders the rows for cache reuse. */
int pn2_fp_apply(const float* dist, const int32_t* idx, const void* unknown_grid,
                 const float* points1, int C1, const float* points2, int C2, int B, int n, int m,
                 float* out, pn2_stream_t stream);
/* pn2_fp_fused for a large search (FP4: n = 8192 unknowns, m = 1024 known) in ONE launch:
 * every workgroup sorts the cloud's m known points into a grid in its own LDS (the automatic
 * edge of pn2_grid_build) and searches it, then writes its rows -- the output of
 * pn2_grid_build + pn2_three_nn_grid + pn2_fp_apply, bit for bit. 1 <= m <= 4096 (else
 * PN2_EINVAL); PN2_ENOTSUP when the known grid does not fit this device's LDS per workgroup
 * (use those three). `unknown_grid` (optional, a grid over the n unknown points)
 * orders the rows as in pn2_fp_apply; with it xyz1 may be NULL. dist / idx (B,n,3): the
 * three_nn result as well, or both NULL. C1 + C2 >= 1. */
int pn2_fp_grid_fused(const float* xyz1, const float* xyz2, const void* unknown_grid,
                      const float* points1, int C1, const float* points2, int C2, int B, int n,
                      int m, float* out, float* dist, int32_t* idx, pn2_stream_t stream);
/* pn2_fp_grid_fused from a grid of the known points built before (known_grid =
 * pn2_grid_build(xyz2, B, m, 0, ...) or pn2_fps_chain_grid's grid0): each workgroup copies
 * its cloud's grid into LDS instead of sorting xyz2 itself. The same output, bit for bit. A
 * grid with more than max(m, 64) cells (an explicit edge) is not staged: the workgroups then
 * build their own from xyz2, which is therefore always required. */
int pn2_fp_grid_fused_known(const void* known_grid, const float* xyz1, const float* xyz2,
                            const void* unknown_grid, const float* points1, int C1,
                            const float* points2, int C2, int B, int n, int m, float* out,
                            float* dist, int32_t* idx, pn2_stream_t stream);

/* ---------------------------------------------------------------- attention / pooling --- */

/* AttentionLayer reduction core (attention_layer.py:35-42) with key_dim = output_dim = 4,
 * heads H = C/4. Q (B,M,C), K,V (B,M,ns,C) → out (B,M,C). Head h reads the CONTIGUOUS
 * block [4*ns*h, 4*ns*(h+1)) of each group's flattened ns*C K/V values as ns rows of 4
 * (the reference's tf.reshape reinterpretation), s = (K_h·q_h)/2, a = softmax(s),
 * out[4h:4h+4] = aᵀ V_h. C must be a multiple of 4. */
int pn2_attn_reduce(const float* Q, const float* K, const float* V, int B, int M, int ns,
                    int C, float* out, pn2_stream_t stream);
/* Several attention reductions of one nsample in ONE launch (the SSG stack's four SA layers,
 * attention_layer.py:35-42 per layer): per layer exactly pn2_attn_reduce(Q, K, V, B, M, ns,
 * C, out); one nsample for every layer, else PN2_EINVAL (an nsample outside {8, 16, 32, 64, 128},
 * or a layer too large for the one-launch task arithmetic, runs as pn2_attn_reduce does). */
#define PN2_ATTN_MAX_LAYERS 4
typedef struct pn2_attn_layer {
  const float* Q;
  const float* K;
  const float* V;
  int M, ns, C;
  float* out;
} pn2_attn_layer;
int pn2_attn_reduce_layers(const pn2_attn_layer* layers, int nlayers, int B,
                           pn2_stream_t stream);
/* Backward of pn2_attn_reduce (TF autodiff of attention_layer.py:35-42): grad_Q (B,M,C),
 * grad_K / grad_V (B,M,ns,C) from grad_out (B,M,C). Every element written (no accumulation);
 * 16-byte aligned buffers, C % 4 == 0. */
int pn2_attn_reduce_grad(const float* Q, const float* K, const float* V, const float* grad_out,
                         int B, int M, int ns, int C, float* grad_Q, float* grad_K,
                         float* grad_V, pn2_stream_t stream);
/* Per-group pooling over nsample (pointnet_util.py:130-145): x (B,M,ns,C) → out (B,M,C),
 * or (B,M,2C) = [avg, max] for PN2_POOL_MAX_AND_AVG. grouped_xyz (B,M,ns,3) is read only
 * by PN2_POOL_WEIGHTED_AVG (w = exp(-5|xyz|)/sum). */
int pn2_group_pool(const float* x, const float* grouped_xyz, int B, int M, int ns, int C,
                   int mode, float* out, pn2_stream_t stream);

/* ---------------------------------------------------------------- shared MLP ------------ */

/* One 1x1-conv layer of tf_util.conv2d / conv1d in inference mode (tf_util.py:165-185):
 *   y[o] = act(((sum_f x[f] * weight[f][o]) + bias[o]) * bn_scale[o] + bn_shift[o])
 * with bn_scale = gamma / sqrt(moving_var + eps), bn_shift = beta - moving_mean * bn_scale
 * (tf.contrib.layers.batch_norm, is_training=False; tf_util.py:512-531). weight (cin,cout)
 * is TF's [1,1,cin,cout] kernel, row-major. bias, bn_scale, bn_shift (cout) may be NULL
 * (bn_scale and bn_shift together). Packs into `packed` (pn2_mlp_packed_size bytes, 16-byte
 * aligned device memory); stored as scale and (bias*scale + shift). */
size_t pn2_mlp_packed_size(int cin, int cout);
int pn2_mlp_pack(const float* weight, const float* bias, const float* bn_scale,
                 const float* bn_shift, int cin, int cout, void* packed, size_t packed_bytes,
                 pn2_stream_t stream);

/* pointnet_sa_module after sampling and ball query (pointnet_util.py:106-145, MSG :184-200):
 * group + centre + concat exactly as pn2_group_concat (flags), then `nlayers` packed layers
 * (layers[0].cin = the grouped width; layers[i+1].cin = layers[i].cout), then pooling over the
 * nsample neighbours:
 *   pool = PN2_POOL_MAX / AVG / WEIGHTED_AVG → out (B,M,cout); PN2_POOL_MAX_AND_AVG →
 *   (B,M,2*cout) = [avg, max]; PN2_POOL_NONE → out (B,M,nsample,cout) (the per-point
 *   features the attention SA modules feed to AttentionLayer, attention_layer.py:229-263).
 * Products and sums in fp32 on the matrix cores; the grouped input and the per-layer
 * activations stay on chip. Host array `layers`. */
int pn2_group_mlp(const float* xyz, const float* points, const float* new_xyz,
                  const int32_t* idx, int B, int N, int C, int M, int nsample, int flags,
                  int nlayers, const pn2_mlp_layer* layers, int pool, float* out,
                  pn2_stream_t stream);
/* pointnet_sa_module_attention (attention_layer.py:229-276) after sampling and ball query:
 * group + MLP as pn2_group_mlp, then — without the per-point features leaving the chip — the
 * AttentionLayer (attention_layer.py:10-45, output_dim = key_dim = 4, heads = C/4):
 * qkv[0..2] = the packed Dense query / key / value layers (C -> C, no activation;
 * pn2_mlp_pack with the Dense kernel and bias), query = the group's first neighbour (:259),
 * head h = the flat block [4*ns*h, 4*ns*(h+1)) of the group's (ns, C) keys and values (the
 * tf.reshape of :35-36), softmax((K_h q_h)/2) V_h; then the inference batch norm
 * out = att * bn_scale + bn_shift (:261; NULL = none) and, with add_max, + the max over nsample
 * of the MLP output (pointnet_sa_module_attention_and_pooling, :296-303). out (B,M,C).
 * nsample <= 128; C = layers[nlayers-1].cout, a multiple of 32. */
int pn2_group_mlp_attention(const float* xyz, const float* points, const float* new_xyz,
                            const int32_t* idx, int B, int N, int C, int M, int nsample,
                            int flags, int nlayers, const pn2_mlp_layer* layers,
                            const pn2_mlp_layer* qkv, const float* bn_scale,
                            const float* bn_shift, int add_max, float* out,
                            pn2_stream_t stream);
/* pointnet_fp_module (pointnet_util.py:218-238): IDW weights of dist (B,n,3) + interpolation
 * of points2 (B,m,C2) at nn_idx (B,n,3) + concat [interp, points1 (B,n,C1)] (bit-identical to
 * pn2_fp_apply's output) fed to the packed layers → out (B,n,cout). points1 may be NULL
 * (C1 = 0). dist / nn_idx come from pn2_three_nn or pn2_three_nn_grid. */
int pn2_fp_mlp(const float* dist, const int32_t* nn_idx, const float* points1, int C1,
               const float* points2, int C2, int B, int n, int m, int nlayers,
               const pn2_mlp_layer* layers, float* out, pn2_stream_t stream);
/* Per-point MLP over rows: x (rows,cin) → out (rows,cout) (tf_util.conv1d with kernel 1,
 * e.g. the fc1/fc2 head of pointnet2_sem_seg.py:57-60). */
int pn2_shared_mlp(const float* x, long long rows, int cin, int nlayers,
                   const pn2_mlp_layer* layers, float* out, pn2_stream_t stream);

/* ---------------------------------------------------------------- scene crops ---------- */

/* Scene bounding box: bbox = [min x, min y, min z, max x, max y, max z] of points (N,3)
 * (reduce_min / reduce_max, data_transformation.py:90-91). workspace:
 * pn2_scene_workspace_size(N) bytes of device memory. */
size_t pn2_scene_workspace_size(int N);
int pn2_scene_bbox(const float* points, int N, float* bbox, void* workspace,
                   size_t workspace_bytes, pn2_stream_t stream);
/* get_subset (data_transformation.py:70-154) for B crops of one scene, with the reference's
 * random draws supplied by the caller: centres (B,T) = the point index each try is centred on
 * (:95-97, T = 10 in the reference), u (B,K) = the uniform [0,1) draws of the final choice
 * (:146). Try t's area: x, y within the centre -+ 0.75, z over the scene (:98-103); points
 * inside it +0.2 (>= lo, < hi) in index order; valid if labelled / (3 n) >= 0.7 (the
 * reference divides by reduce_sum(ones_like((n,3) points)), :113) and the occupied voxel keys
 * / 31 / 31 / 62 >= 0.02 (:119-126); the first valid try is kept, else the last (:138-141).
 * With the 3 n denominator no try can be valid (labelled / 3n <= 1/3), so the last try is
 * used without evaluating the others; the earlier centres only mirror the reference's draws.
 * Outputs (B,K[,3]): points, labels, colors (int32, may be NULL with out_colors NULL),
 * normals (may be NULL likewise), weights = label_weights[label] * mask, mask = inside the
 * area +0.01 (:114-117, :150-153). bbox from pn2_scene_bbox. workspace:
 * pn2_crop_workspace_size(B, N, T) bytes. */
size_t pn2_crop_workspace_size(int B, int N, int T);
int pn2_crop_sample(const float* points, const int32_t* labels, const int32_t* colors,
                    const float* normals, int N, const float* bbox, const int32_t* centres,
                    int B, int T, const float* u, int K, const float* label_weights, int nlw,
                    void* workspace, size_t workspace_bytes, float* out_points,
                    int32_t* out_labels, int32_t* out_colors, float* out_normals,
                    float* out_weights, pn2_stream_t stream);
/* Whole-scene chunker, selection part (complete_scene_loader.py:33-40): for each of S boxes
 * bounds (S,6) = [lo xyz, hi xyz] in FLOAT64 (the reference's float32 points compare against
 * float64 bounds), the indices of the points with lo - margin <= p <= hi + margin on all axes,
 * ascending, in sel[s*N ...], inner[s*N + k] = 1 if that point is also within [lo, hi], and the
 * per-slice counts in counts (S, pn2_subvolume_slices(N)) — their row sums are the subvolume
 * sizes. The random shuffle / fill-up of the chunks is drawn by the caller. */
int pn2_subvolume_slices(int N);
int pn2_subvolume_select(const float* points, int N, const double* bounds, int S, double margin,
                         int32_t* counts, int32_t* sel, uint8_t* inner, pn2_stream_t stream);
/* dst[r] = src[idx[r]] for n rows of row_bytes bytes (a multiple of 4); idx outside
 * [0, nsrc) reads row 0. */
int pn2_gather_rows(const void* src, long long nsrc, int row_bytes, const int32_t* idx,
                    long long n, void* dst, pn2_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* PN2HIP_H */
