// Shared point-wise MLP (1x1 conv + bias + inference batch norm + ReLU) fused with the step
// before it (grouping, or three-point interpolation) and the pooling after it, gfx950.
//
// Replaces, per SA layer, the TF graph of pointnet_util.py:106-145 (pointnet_sa_module):
//   sample_and_group's grouped [xyz - new_xyz, points]  (pointnet_util.py:39-56, MSG :186-193)
//   -> for each mlp width: tf_util.conv2d(1x1) = conv + bias_add + batch_norm + relu
//      (tf_util.py:165-185, batch_norm_template :512-531, inference mode)
//   -> reduce_max / reduce_mean / weighted_avg / max_and_avg over nsample (:130-145, :200)
// and per FP layer pointnet_fp_module's interpolation + concat + MLP (pointnet_util.py:218-238),
// plus plain per-point MLPs (the conv1d head fc1/fc2, pointnet2_sem_seg.py:57-60).
//
// Design: one workgroup owns P = 32*R point rows (whole groups, or one slice
// of a group larger than P). The rows' input features are gathered ONCE into LDS; every layer
// then runs from LDS to LDS on the fp32 matrix cores (v_mfma_f32_32x32x2_f32: exact fp32
// products, fp32 accumulation — TF's conv2d is fp32 too), and the last layer is pooled in
// registers, so the (rows x width) activations never touch HBM. The reference materialises
// new_points (B,M,ns,3+C) and every layer's output in HBM.
//
// MFMA orientation. For layer outputs that feed another layer the product is computed as
// Y^T = W^T X^T (A = weights: output feature on the lane, B = activations: point on the lane):
// the accumulator's rows are 4 consecutive features per register quad, stored to LDS as one
// 16-byte write per quad. The LAST layer swaps A and B (Y = X W): the accumulator holds 16 of
// the tile's 32 points per lane for one output feature, so pooling over a group is a register
// max/sum plus one lane^32 exchange, and per-point outputs are 128-byte row segments.
// Both orientations read the operands through the same lane maps, so one packed weight format
// serves every layer: Wp[to][c][h][i][s] = W[8c + 4h + s][32*to + i] (pn2_mlp_pack), one
// float4 per lane per 4 MFMAs, and activations are read as act[p][8c + 4h .. +3].
#include <cstdio>
#include <cstdlib>

#include "common.h"

namespace pn2 {
namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / kWave;
constexpr int kMaxGroupsPerWG = 16;  // P / ns_pad with P <= 128, ns_pad >= 8

enum Src : int { kSrcGroup = 0, kSrcFP = 1, kSrcRows = 2 };
enum Layout : int { kPointsOnly = 0, kXyzOnly = 1, kXyzFirst = 2, kXyzLast = 3 };

struct LayerDev {
  const float4* w;     // packed weights [cout32][cin8][64] float4
  const float* scale;  // [cout32*32]
  const float* shift;  // [cout32*32]
  int cin8, cout32, cout, relu;
  int lofs;  // float offset of this layer's packed block in the LDS weight copy (WL kernels)
};

struct Params {
  LayerDev L[PN2_MLP_MAX_LAYERS];
  int nl;
  int width0;            // layer-0 input width in LDS (cin8*8)
  int stride0, stride1;  // LDS row strides (floats) of the activation buffers
  int off1, off_part, off_run, off_meta;  // float offsets into dynamic LDS
  int off_w, wfloats;  // WL kernels: LDS copy of every layer's packed block (wfloats floats)
  int direct_pool;     // one pass, ns_pad <= 32: a row tile's pooled values are final
  // input row = segment A (+ segment B) (+ zero padding up to width0); nA/nB = units per row
  // (float4 chunks when vecA/vecB, else floats), offA/offB = LDS column of the segment
  int nA, nB, offA, offB, vecA, vecB, cin_total;
  FastDiv divA, divB, div_pad;
  // group source
  const float* xyz;
  const float* points;
  const float* new_xyz;
  const int32_t* idx;
  int N, C, M, ns, lg_ns_pad, layout, ngroups, passes, gpw;
  // fp source
  const float* dist;
  const int32_t* nn;
  const float* p1;
  const float* p2;
  int C1, C2, n, m;
  // rows source
  const float* x;
  int cin;
  long long rows;
  int pool;
  float* out;
  unsigned long long* stamp;  // PN2_MLP_STAMP builds: per-workgroup phase timestamps
  // attention tail (pn2_group_mlp_attention): the MLP's last layer stays in LDS (X), then the
  // Dense query (first neighbour of each group) / key / value layers, the reduction per head
  // and the batch norm (+ max pool of X), column segment by column segment of K and V
  int attn, att_wseg, att_nseg, att_add_max;
  int stage_out;  // rows / fp sources: the last layer goes to LDS, then whole rows to HBM
  int out_vec;    // stage_out with cout % 4 == 0 and a 16-byte aligned out: float4 stores
  int ntiles;  // tiles of P rows
  int tpw;     // consecutive tiles per workgroup (grid = ceil(ntiles / tpw))
  LayerDev qkv[3];
  const float* att_scale;
  const float* att_shift;
  int off_k, off_v, off_q, stride_kv, stride_q;
};

#ifdef PN2_MLP_STAMP
// s_memtime at phase boundaries of the first kStampWG workgroups (wave 0), slot k of 16
constexpr int kStampWG = 4096;
#define PN2_STAMP(k)                                                                    \
  do {                                                                                 \
    if (prm.stamp && blockIdx.x < kStampWG && threadIdx.x == 0)                        \
      prm.stamp[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime();                 \
  } while (0)
unsigned long long* g_stamp = nullptr;
#else
#define PN2_STAMP(k) \
  do {               \
  } while (0)
#endif

PN2_DEV float act(float v, int relu) { return relu ? fmaxf(v, 0.f) : v; }

// weight = (1/d)/sum(1/d), d = max(dist, 1e-10)  (pointnet_util.py:219-222); same fp32 order
// as interp.hip's idw(), so the interpolated features are bit-identical to pn2_fp_apply's.
PN2_DEV void idw3(float d1, float d2, float d3, float& w1, float& w2, float& w3) {
  const float r1 = 1.0f / fmaxf(d1, 1e-10f);
  const float r2 = 1.0f / fmaxf(d2, 1e-10f);
  const float r3 = 1.0f / fmaxf(d3, 1e-10f);
  const float norm = (r1 + r2) + r3;
  w1 = r1 / norm;
  w2 = r2 / norm;
  w3 = r3 / norm;
}


// One output tile over RG row tiles: cin8 chunks of 8 input features, 4 MFMAs per chunk and
// row tile (k = 8c + 4h + s, s = 0..3); every weight fragment serves the RG row tiles'
// independent accumulators. wp = the tile's packed weights at this lane, ap = this lane's
// activation row (+4h) in the first row tile, rstride = floats between row tiles. Chunks run
// in groups of G with the next group's weights and activations loaded (and pinned there by
// sched_barrier) before the current group's MFMAs are issued; the last group re-loads itself
// (branch-free), then a remainder of single chunks.
// LAST: Y = X W (points in the accumulator rows) instead of Y^T = W^T X^T.
template <bool LAST, int RG>
PN2_DEV void mma_item(const float4* __restrict__ wp, const float* ap, int rstride, int cin8,
                      f32x16 (&acc)[RG]) {
  constexpr int G = RG >= 2 ? 2 : 4;  // 16 MFMAs (~1000 cycles) per group either way
#pragma unroll
  for (int r = 0; r < RG; ++r)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[r][i] = 0.f;
  auto mma4 = [&](const float4& w, const float4& a, f32x16& c) {
    if (LAST) {
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, w.x, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, w.y, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, w.z, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, w.w, c, 0, 0, 0);
    } else {
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(w.x, a.x, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(w.y, a.y, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(w.z, a.z, c, 0, 0, 0);
      c = __builtin_amdgcn_mfma_f32_32x32x2f32(w.w, a.w, c, 0, 0, 0);
    }
  };
  auto act4 = [&](int r, int c) {
    return *reinterpret_cast<const float4*>(ap + r * rstride + 8 * c);
  };
  const int cg = cin8 - cin8 % G;
  float4 wA[G], aA[G][RG], wB[G], aB[G][RG];
  auto load = [&](float4* w, float4 (*a)[RG], int c) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      w[u] = wp[(size_t)(c + u) * kWave];
#pragma unroll
      for (int r = 0; r < RG; ++r) a[u][r] = act4(r, c + u);
    }
  };
  auto compute = [&](const float4* w, float4 (*a)[RG]) {
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
      for (int r = 0; r < RG; ++r) mma4(w[u], a[u][r], acc[r]);
  };
  if (cg > 0) {
    load(wA, aA, 0);
    for (int c = 0; c < cg; c += 2 * G) {
      const bool two = c + G < cg;
      load(wB, aB, two ? c + G : c);
      __builtin_amdgcn_sched_barrier(0);
      compute(wA, aA);
      __builtin_amdgcn_sched_barrier(0);
      if (!two) break;
      load(wA, aA, c + 2 * G < cg ? c + 2 * G : c);
      __builtin_amdgcn_sched_barrier(0);
      compute(wB, aB);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  for (int c = cg; c < cin8; ++c) {
    const float4 w = wp[(size_t)c * kWave];
#pragma unroll
    for (int r = 0; r < RG; ++r) mma4(w, act4(r, c), acc[r]);
  }
}

// One segment of every slot's input row: n units per row (float4 chunks or floats), fetched
// by fetch(p, j) and stored at LDS column off + j*units. Batches of kGatherUnroll independent
// units per thread: every load of a batch is issued before the first LDS store, so the L2/HBM
// latency is paid once per batch.
template <typename T, int P, typename F>
PN2_DEV void gather_segment(int n, FastDiv div_n, int off, float* act, int stride, F fetch) {
  constexpr int V = sizeof(T) / sizeof(float);
  constexpr int kGatherUnroll = V == 4 ? 4 : 8;
  const int total = P * n;
  for (int e0 = threadIdx.x; e0 < total; e0 += kBlock * kGatherUnroll) {
    T vals[kGatherUnroll];
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int e = min(e0 + u * kBlock, total - 1);  // branch-free: every load in flight
      const int p = (int)fdiv((uint32_t)e, div_n);
      vals[u] = fetch(p, e - p * n);
    }
#pragma unroll
    for (int u = 0; u < kGatherUnroll; ++u) {
      const int e = e0 + u * kBlock;
      if (e < total) {
        const int p = (int)fdiv((uint32_t)e, div_n);
        float* dst = act + p * stride + off + V * (e - p * n);
        if constexpr (V == 4) {
          if ((off & 3) == 0) {
            *reinterpret_cast<float4*>(dst) = vals[u];
          } else {
            dst[0] = vals[u].x;
            dst[1] = vals[u].y;
            dst[2] = vals[u].z;
            dst[3] = vals[u].w;
          }
        } else {
          *dst = vals[u];
        }
      }
    }
  }
}

PN2_DEV float4 f4mul(float4 a, float w) { return make_float4(a.x * w, a.y * w, a.z * w, a.w * w); }
PN2_DEV float4 f4add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

// The input rows of the workgroup's P slots into act0 [P][width0]: the source's segments
// then zeros up to width0.
template <int SRC, int P>
PN2_DEV void gather_rows(const Params& prm, float* act0, const int* s_src, const int* s_aux,
                         const float* s_fw, const int* s_fi) {
  const int S = prm.stride0;
  if (SRC == kSrcGroup) {
    // grouped points rows, then the centred xyz (pointnet_util.py:39-56 / :186-193)
    const float* pts = prm.points;
    const int C = prm.C;
    if (prm.nA) {
      if (prm.vecA)
        gather_segment<float4, P>(prm.nA, prm.divA, prm.offA, act0, S, [&](int p, int j) {
          const int src = s_src[p];
          return src < 0 ? make_float4(0.f, 0.f, 0.f, 0.f)
                         : *reinterpret_cast<const float4*>(pts + (size_t)src * C + 4 * j);
        });
      else
        gather_segment<float, P>(prm.nA, prm.divA, prm.offA, act0, S, [&](int p, int j) {
          const int src = s_src[p];
          return src < 0 ? 0.f : pts[(size_t)src * C + j];
        });
    }
    if (prm.nB)
      gather_segment<float, P>(3, prm.divB, prm.offB, act0, S, [&](int p, int j) {
        const int src = s_src[p];
        // pointnet_util.py:40: fp32 subtraction, bit-exact with pn2_group_concat
        return src < 0 ? 0.f
                       : prm.xyz[(size_t)src * 3 + j] - prm.new_xyz[(size_t)s_aux[p] * 3 + j];
      });
  } else if (SRC == kSrcFP) {
    // interpolation (tf_interpolate.cpp:107-127: ((p1*w1) + (p2*w2)) + (p3*w3)), then points1
    const float* p2 = prm.p2;
    const int C2 = prm.C2;
    if (prm.vecA)
      gather_segment<float4, P>(prm.nA, prm.divA, 0, act0, S, [&](int p, int j) {
        if (s_src[p] < 0) return make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 a = *reinterpret_cast<const float4*>(p2 + (size_t)s_fi[3 * p] * C2 + 4 * j);
        const float4 b = *reinterpret_cast<const float4*>(p2 + (size_t)s_fi[3 * p + 1] * C2 + 4 * j);
        const float4 c = *reinterpret_cast<const float4*>(p2 + (size_t)s_fi[3 * p + 2] * C2 + 4 * j);
        return f4add(f4add(f4mul(a, s_fw[3 * p]), f4mul(b, s_fw[3 * p + 1])),
                     f4mul(c, s_fw[3 * p + 2]));
      });
    else
      gather_segment<float, P>(prm.nA, prm.divA, 0, act0, S, [&](int p, int j) {
        if (s_src[p] < 0) return 0.f;
        const float a = p2[(size_t)s_fi[3 * p] * C2 + j] * s_fw[3 * p];
        const float b = p2[(size_t)s_fi[3 * p + 1] * C2 + j] * s_fw[3 * p + 1];
        const float c = p2[(size_t)s_fi[3 * p + 2] * C2 + j] * s_fw[3 * p + 2];
        return (a + b) + c;
      });
    const float* p1 = prm.p1;
    const int C1 = prm.C1;
    if (prm.nB) {  // concat [interp, points1] (pointnet_util.py:226)
      if (prm.vecB)
        gather_segment<float4, P>(prm.nB, prm.divB, prm.offB, act0, S, [&](int p, int j) {
          const int src = s_src[p];
          return src < 0 ? make_float4(0.f, 0.f, 0.f, 0.f)
                         : *reinterpret_cast<const float4*>(p1 + (size_t)src * C1 + 4 * j);
        });
      else
        gather_segment<float, P>(prm.nB, prm.divB, prm.offB, act0, S, [&](int p, int j) {
          const int src = s_src[p];
          return src < 0 ? 0.f : p1[(size_t)src * C1 + j];
        });
    }
  } else {
    const float* x = prm.x;
    const int cin = prm.cin;
    if (prm.vecA)
      gather_segment<float4, P>(prm.nA, prm.divA, 0, act0, S, [&](int p, int j) {
        const int src = s_src[p];
        return src < 0 ? make_float4(0.f, 0.f, 0.f, 0.f)
                       : *reinterpret_cast<const float4*>(x + (size_t)src * cin + 4 * j);
      });
    else
      gather_segment<float, P>(prm.nA, prm.divA, 0, act0, S, [&](int p, int j) {
        const int src = s_src[p];
        return src < 0 ? 0.f : x[(size_t)src * cin + j];
      });
  }
  const int npad = prm.width0 - prm.cin_total;
  if (npad > 0)
    for (int e = threadIdx.x; e < P * npad; e += kBlock) {
      const int p = (int)fdiv((uint32_t)e, prm.div_pad);
      act0[p * S + prm.cin_total + (e - p * npad)] = 0.f;
    }
}

// Row-tile groups per layer: at most kMaxRG row tiles share an item (register budget of two
// waves per SIMD), and layers narrower than the 4 waves split further so every wave works.
constexpr int kMaxRG = 2;
__host__ __device__ inline int item_split(int R, int c32) {
  int nsplit = R > kMaxRG ? R / kMaxRG : 1;
  while (nsplit < R && nsplit * c32 < kWaves) nsplit <<= 1;
  return nsplit;
}

// pooled output of group g, feature fo (pointnet_util.py:130-145)
PN2_DEV void store_pooled(const Params& prm, int g, int fo, int cout, float mx, float sm) {
  const float avg = sm / (float)prm.ns;
  if (prm.pool == PN2_POOL_MAX) prm.out[(size_t)g * cout + fo] = mx;
  else if (prm.pool == PN2_POOL_AVG) prm.out[(size_t)g * cout + fo] = avg;
  else if (prm.pool == PN2_POOL_WEIGHTED_AVG) prm.out[(size_t)g * cout + fo] = sm;
  else {  // max_and_avg: concat [avg, max] (pointnet_util.py:145)
    prm.out[(size_t)g * 2 * cout + fo] = avg;
    prm.out[(size_t)g * 2 * cout + cout + fo] = mx;
  }
}

// One Dense layer item (no activation) of the attention tail: output tile `to` of layer D
// over row tile rt of X, written (scale/shift epilogue = bias) into dst at column
// (to - to0)*32, rows 32*rt + col. For the query, row_of_lane maps lane col to X row
// col*ns_pad (the first neighbour of group col) and only rows < nrows are written.
template <int RG>
PN2_DEV void dense_item(const LayerDev& D, const float* X, int Sx, int xrow, int to, int to0,
                        float* dst, int Sd, int drow, int lane, int h) {
  float4 sc[4], sh[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int fb = 32 * to + 8 * q + 4 * h;
    sc[q] = *reinterpret_cast<const float4*>(D.scale + fb);
    sh[q] = *reinterpret_cast<const float4*>(D.shift + fb);
  }
  f32x16 acc[RG];
  mma_item<false, RG>(D.w + (size_t)to * D.cin8 * kWave + lane, X + xrow * Sx + 4 * h, 32 * Sx,
                      D.cin8, acc);
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    float* op = dst + (drow + 32 * r) * Sd + 32 * (to - to0) + 4 * h;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float4 y;
      y.x = acc[r][4 * q + 0] * sc[q].x + sh[q].x;
      y.y = acc[r][4 * q + 1] * sc[q].y + sh[q].y;
      y.z = acc[r][4 * q + 2] * sc[q].z + sh[q].z;
      y.w = acc[r][4 * q + 3] * sc[q].w + sh[q].w;
      *reinterpret_cast<float4*>(op + 8 * q) = y;
    }
  }
}

// (1x4)·(4x1) of tf.matmul, summed left to right (as attn.hip)
PN2_DEV float dot4q(float4 q, float4 k) {
  float s = q.x * k.x;
  s = s + q.y * k.y;
  s = s + q.z * k.z;
  s = s + q.w * k.w;
  return s;
}

// The query of every group, Dense_q(X[first neighbour]) (attention_layer.py:31, :259), on the
// VALU: only G rows are needed, so a 32-row MFMA tile would waste (32 - G)/32 of its work
// (31/32 at SA3/SA4, where one group fills the workgroup). Thread -> (group, output feature);
// the packed weights are read as one float4 over 4 consecutive input features, the row of X
// as LDS broadcasts. Four partial sums (one per feature residue mod 4), then the epilogue.
PN2_DEV void attn_query(const LayerDev& D, const float* X, int Sx, int G, int ns_pad, float* Qb,
                        int Sq, int C) {
  for (int o = threadIdx.x; o < G * C; o += kBlock) {
    const int gi = o / C, f = o - gi * C;
    const float4* wp = D.w + (size_t)(f >> 5) * D.cin8 * kWave + (f & 31);
    const float* x = X + gi * ns_pad * Sx;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 4
    for (int c = 0; c < D.cin8; ++c) {
      const float4 w0 = wp[c * kWave], w1 = wp[c * kWave + 32];
      const float4 x0 = *reinterpret_cast<const float4*>(x + 8 * c);
      const float4 x1 = *reinterpret_cast<const float4*>(x + 8 * c + 4);
      a0 = fmaf(x0.x, w0.x, a0);
      a1 = fmaf(x0.y, w0.y, a1);
      a2 = fmaf(x0.z, w0.z, a2);
      a3 = fmaf(x0.w, w0.w, a3);
      a0 = fmaf(x1.x, w1.x, a0);
      a1 = fmaf(x1.y, w1.y, a1);
      a2 = fmaf(x1.z, w1.z, a2);
      a3 = fmaf(x1.w, w1.w, a3);
    }
    Qb[gi * Sq + f] = ((a0 + a1) + (a2 + a3)) * D.scale[f] + D.shift[f];
  }
}

template <int L>
PN2_DEV float lane_sum(float v) {
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v = v + __shfl_xor(v, o, kWave);
  return v;
}
template <int L>
PN2_DEV float lane_max(float v) {
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

// Scores, softmax over the ns pseudo-keys and the weighted V of every (group, head) unit of
// one K/V column segment (attention_layer.py:37-40) [+ the batch norm of :261 and the max pool
// of :296-303], L lanes per unit: each lane takes every L-th pseudo-key, so the per-unit sums
// are register sums plus log2(L) lane exchanges (L is picked so the units fill the block).
template <int L>
PN2_DEV void attn_scores(const Params& prm, const float* X, int Sx, const float* Kb,
                         const float* Vb, const float* Qb, int sgi, int tile) {
  const int C = prm.L[prm.nl - 1].cout;
  const int ns = prm.ns, ns_pad = 1 << prm.lg_ns_pad;
  const int G = prm.gpw;
  const int Skv = prm.stride_kv, Sq = prm.stride_q;
  const int wseg = prm.att_wseg;
  const bool whole = wseg == C;
  const int hs_per_group = whole ? C / 4 : ns;  // heads completed by one segment
  const int units = G * hs_per_group;
  const int sub = threadIdx.x & (L - 1);
  for (int u = threadIdx.x / L; u < units; u += kBlock / L) {
    const int gi = u / hs_per_group, hs = u - gi * hs_per_group;
    const int g = tile * G + gi;
    const int hg = whole ? hs : (C / wseg) * hs + sgi;  // the head's index in [0, C/4)
    const float4 q = *reinterpret_cast<const float4*>(Qb + gi * Sq + 4 * hg);
    const int r0 = gi * ns_pad;
    auto key_at = [&](int j, const float* B) {
      int row, c;
      if (whole) {
        const int f = 4 * ns * hs + 4 * j;  // flat index in the group's (ns, C) matrix
        row = f / C;
        c = f - row * C;
      } else {
        row = hs;
        c = 4 * j;
      }
      return *reinterpret_cast<const float4*>(B + (r0 + row) * Skv + c);
    };
    float mx = -__builtin_inff();
    for (int j = sub; j < ns; j += L) mx = fmaxf(mx, dot4q(q, key_at(j, Kb)) / 2.0f);
    mx = lane_max<L>(mx);  // softmax (:39)
    float sum = 0.f;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int j = sub; j < ns; j += L) {
      const float e = expf(dot4q(q, key_at(j, Kb)) / 2.0f - mx);
      sum = sum + e;
      const float4 v = key_at(j, Vb);
      o.x = o.x + e * v.x;
      o.y = o.y + e * v.y;
      o.z = o.z + e * v.z;
      o.w = o.w + e * v.w;
    }
    sum = lane_sum<L>(sum);
    o.x = lane_sum<L>(o.x) / sum;  // aᵀ·V_h (:40), a = e / sum
    o.y = lane_sum<L>(o.y) / sum;
    o.z = lane_sum<L>(o.z) / sum;
    o.w = lane_sum<L>(o.w) / sum;
    float4 pm = make_float4(0.f, 0.f, 0.f, 0.f);
    if (prm.att_add_max) {  // + reduce_max over ns of X (:296-303)
      float4 m4 = make_float4(-__builtin_inff(), -__builtin_inff(), -__builtin_inff(),
                              -__builtin_inff());
      for (int j = sub; j < ns; j += L) {
        const float4 x = *reinterpret_cast<const float4*>(X + (r0 + j) * Sx + 4 * hg);
        m4.x = fmaxf(m4.x, x.x);
        m4.y = fmaxf(m4.y, x.y);
        m4.z = fmaxf(m4.z, x.z);
        m4.w = fmaxf(m4.w, x.w);
      }
      pm = make_float4(lane_max<L>(m4.x), lane_max<L>(m4.y), lane_max<L>(m4.z),
                       lane_max<L>(m4.w));
    }
    if (sub == 0 && g < prm.ngroups) {
      float4 y = o;
      if (prm.att_scale) {  // batch_norm_for_conv2d, inference (:261)
        const float4 s4 = *reinterpret_cast<const float4*>(prm.att_scale + 4 * hg);
        const float4 t4 = *reinterpret_cast<const float4*>(prm.att_shift + 4 * hg);
        y = make_float4(y.x * s4.x + t4.x, y.y * s4.y + t4.y, y.z * s4.z + t4.z,
                        y.w * s4.w + t4.w);
      }
      if (prm.att_add_max) y = make_float4(y.x + pm.x, y.y + pm.y, y.z + pm.z, y.w + pm.w);
      *reinterpret_cast<float4*>(prm.out + (size_t)g * C + 4 * hg) = y;
    }
  }
}

// AttentionLayer.call (attention_layer.py:29-45) + batch_norm_for_conv2d (:261) [+ the max pool
// of :296-303] on the workgroup's groups, from the MLP output X (P rows x C) in LDS.
// Head h of a group reads the flat block [4*ns*h, 4*ns*(h+1)) of the group's row-major (ns, C)
// K and V (the tf.reshape quirk of :35-36): with C <= 4*ns that block spans whole rows (K and V
// are computed whole, one segment); with C = k*4*ns it is the column block h % k of row h / k,
// so K and V are computed k column segments at a time and each segment completes its heads.
template <int R>
PN2_DEV void attention_tail(const Params& prm, float* smem, const float* X, int Sx, int tile) {
  const int tid = threadIdx.x, lane = lane_id(), wave = tid / kWave;
  const int col = lane & 31, h = lane >> 5;
  const int C = prm.L[prm.nl - 1].cout;
  const int G = prm.gpw;
  float* Kb = smem + prm.off_k;
  float* Vb = smem + prm.off_v;
  float* Qb = smem + prm.off_q;
  const int Skv = prm.stride_kv;
  attn_query(prm.qkv[0], X, Sx, G, 1 << prm.lg_ns_pad, Qb, prm.stride_q, C);
  PN2_STAMP(9);
  const int t_seg = prm.att_wseg / 32;
  const int units = G * (prm.att_wseg == C ? C / 4 : prm.ns);
  int L = 32;  // lanes per unit: the largest power of two <= 32 that keeps the units in one pass
  while (L > 1 && units * L > kBlock) L >>= 1;
  while (L > 1 && L > prm.ns) L >>= 1;
  for (int sgi = 0; sgi < prm.att_nseg; ++sgi) {
    // K and V of this column segment (:32-33)
    // items of two row tiles (R >= 2): each weight fragment serves both tiles
    constexpr int RGk = R >= 2 ? 2 : 1;
    constexpr int npair = R / RGk;
    const int nitems = 2 * npair * t_seg;
    for (int item = wave; item < nitems; item += kWaves) {
      const int which = item / (npair * t_seg);
      const int rem = item - which * (npair * t_seg);
      const int to = sgi * t_seg + rem / npair, rt = (rem % npair) * RGk;
      dense_item<RGk>(prm.qkv[1 + which], X, Sx, 32 * rt + col, to, sgi * t_seg,
                      which ? Vb : Kb, Skv, 32 * rt + col, lane, h);
    }
    __syncthreads();
    if (sgi == 0) PN2_STAMP(13);
    switch (L) {
      case 32: attn_scores<32>(prm, X, Sx, Kb, Vb, Qb, sgi, tile); break;
      case 16: attn_scores<16>(prm, X, Sx, Kb, Vb, Qb, sgi, tile); break;
      case 8: attn_scores<8>(prm, X, Sx, Kb, Vb, Qb, sgi, tile); break;
      case 4: attn_scores<4>(prm, X, Sx, Kb, Vb, Qb, sgi, tile); break;
      case 2: attn_scores<2>(prm, X, Sx, Kb, Vb, Qb, sgi, tile); break;
      default: attn_scores<1>(prm, X, Sx, Kb, Vb, Qb, sgi, tile); break;
    }
    __syncthreads();  // the next segment overwrites K and V
    if (sgi == 0) PN2_STAMP(14);
  }
}

// What a layer item needs from the kernel (LDS carve, lane coordinates, pooling state).
struct Ctx {
  const Params* prm;
  const float* wl;  // LDS weight copy (WL kernels) or nullptr
  float* act0;
  float* act1;
  float* part;
  const int* s_src;
  const int* s_aux;
  const float* s_pw;
  int lane, col, h, ns_pad, coutp;
  bool pooled;
  int tile;  // the workgroup's current tile (a workgroup loops over prm.tpw tiles)
};

// One item of layer l: the MFMA product, then either the intermediate epilogue (scale,
// shift, activation, 16-byte writes into the other LDS buffer) or the last layer's (per-point
// stores, or per-group pooling partials in LDS).
template <int SRC, int R, int RG, bool WL>
PN2_DEV void layer_item(const Ctx& cx, int l, bool last, int to, int rt0, int pass) {
  constexpr int P = 32 * R;
  const Params& prm = *cx.prm;
  const LayerDev& Ld = prm.L[l];
  const float4* wbase = Ld.w;
  const float* scale = Ld.scale;
  const float* shift = Ld.shift;
  if (WL) {  // the workgroup's LDS copy of the packed block
    wbase = reinterpret_cast<const float4*>(cx.wl + Ld.lofs);
    scale = cx.wl + Ld.lofs + Ld.cout32 * Ld.cin8 * 256;
    shift = scale + Ld.cout32 * 32;
  }
  const float* in = (l & 1) ? cx.act1 : cx.act0;
  const int Sin = (l & 1) ? prm.stride1 : prm.stride0;
  const int lane = cx.lane, col = cx.col, h = cx.h;
  const float4* wp = wbase + (size_t)to * Ld.cin8 * kWave + lane;
  const float* ap = in + (32 * rt0 + col) * Sin + 4 * h;
  f32x16 acc[RG];
  if (!last) {
    float* outb = (l & 1) ? cx.act0 : cx.act1;
    const int Sout = (l & 1) ? prm.stride0 : prm.stride1;
    // epilogue parameters first: their latency hides under the K loop
    float4 sc[4], sh[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int fb = 32 * to + 8 * q + 4 * h;
      sc[q] = *reinterpret_cast<const float4*>(scale + fb);
      sh[q] = *reinterpret_cast<const float4*>(shift + fb);
    }
    mma_item<false, RG>(wp, ap, 32 * Sin, Ld.cin8, acc);
#pragma unroll
    for (int r = 0; r < RG; ++r) {
      // rows = features 32*to + 8q + 4h + e (e = reg & 3), column = point 32*(rt0+r) + col
      float* op = outb + (32 * (rt0 + r) + col) * Sout + 32 * to + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 y;
        y.x = act(acc[r][4 * q + 0] * sc[q].x + sh[q].x, Ld.relu);
        y.y = act(acc[r][4 * q + 1] * sc[q].y + sh[q].y, Ld.relu);
        y.z = act(acc[r][4 * q + 2] * sc[q].z + sh[q].z, Ld.relu);
        y.w = act(acc[r][4 * q + 3] * sc[q].w + sh[q].w, Ld.relu);
        *reinterpret_cast<float4*>(op + 8 * q) = y;
      }
    }
    return;
  }
  const int fo = 32 * to + col;
  const float s = scale[fo], t = shift[fo];
#ifdef PN2_MLP_STAMP
  const bool st = prm.stamp && blockIdx.x < kStampWG && threadIdx.x == 0 && to == 0;
  if (st) prm.stamp[blockIdx.x * 16 + 10] = __builtin_amdgcn_s_memtime();
#endif
  mma_item<true, RG>(wp, ap, 32 * Sin, Ld.cin8, acc);
#ifdef PN2_MLP_STAMP
  if (st) {
    __builtin_amdgcn_s_waitcnt(0);
    prm.stamp[blockIdx.x * 16 + 11] = __builtin_amdgcn_s_memtime();
  }
#endif
#pragma unroll
  for (int r = 0; r < RG; ++r) {
    const int rt = rt0 + r;
    // rows = points 32*rt + (i&3) + 8(i>>2) + 4h, column = feature fo
    float y[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) y[i] = act(acc[r][i] * s + t, Ld.relu);
    if (!cx.pooled) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int p = 32 * rt + (i & 3) + 8 * (i >> 2) + 4 * h;
        if (cx.s_src[p] < 0 || fo >= Ld.cout) continue;
        long long orow;
        if (SRC == kSrcGroup) {
          // per-point output of the group's k-th neighbour (no pooling)
          const int k = (prm.passes == 1) ? (p & (cx.ns_pad - 1)) : pass * P + p;
          if (k >= prm.ns) continue;
          orow = (long long)cx.s_aux[p] * prm.ns + k;
        } else {
          orow = (long long)cx.tile * P + p;
        }
        prm.out[orow * Ld.cout + fo] = y[i];
      }
    } else {
      // rows of register i: (i&3) + 8(i>>2) + 4h, so register quad q = i>>2 holds rows
      // 8q..8q+7 (both lane halves). Per-quad partials, then groups of 1, 2 or 4 quads
      // (ns_pad 8, 16, >= 32), then the two lane halves (v_permlane32_swap).
      const bool wsum = prm.pool != PN2_POOL_MAX;
      float mq[4], sq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        mq[q] = fmaxf(fmaxf(y[4 * q], y[4 * q + 1]), fmaxf(y[4 * q + 2], y[4 * q + 3]));
        sq[q] = 0.f;
        if (wsum) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            sq[q] = sq[q] + y[4 * q + e] * cx.s_pw[32 * rt + e + 8 * q + 4 * h];
        }
      }
      const int lg = prm.lg_ns_pad;
      int gpt;
      if (lg >= 5) {
        mq[0] = fmaxf(fmaxf(mq[0], mq[1]), fmaxf(mq[2], mq[3]));
        sq[0] = (sq[0] + sq[1]) + (sq[2] + sq[3]);
        gpt = 1;
      } else if (lg == 4) {
        mq[0] = fmaxf(mq[0], mq[1]);
        sq[0] = sq[0] + sq[1];
        mq[1] = fmaxf(mq[2], mq[3]);
        sq[1] = sq[2] + sq[3];
        gpt = 2;
      } else {
        gpt = 4;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < gpt) {
          auto xm = __builtin_amdgcn_permlane32_swap(__float_as_uint(mq[u]),
                                                     __float_as_uint(mq[u]), false, false);
          const float mx = fmaxf(__uint_as_float(xm[0]), __uint_as_float(xm[1]));
          float sm = 0.f;
          if (wsum) {
            auto xs = __builtin_amdgcn_permlane32_swap(__float_as_uint(sq[u]),
                                                       __float_as_uint(sq[u]), false, false);
            sm = __uint_as_float(xs[0]) + __uint_as_float(xs[1]);
          }
          if (prm.direct_pool) {  // this row tile holds whole groups: store the final value
            const int g = cx.tile * prm.gpw + rt * gpt + u;
            if (h == 0 && g < prm.ngroups && fo < Ld.cout)
              store_pooled(prm, g, fo, Ld.cout, mx, sm);
#ifdef PN2_MLP_STAMP
            if (st) prm.stamp[blockIdx.x * 16 + 12] = __builtin_amdgcn_s_memtime();
#endif
          } else if (h == 0) {
            float* pp = cx.part + ((size_t)(rt * 4 + u) * 2) * cx.coutp + fo;
            pp[0] = mx;
            pp[cx.coutp] = sm;
          }
        }
      }
    }
  }
}

// Per-slot metadata in two steps so a multi-tile workgroup can issue the next unit's global
// loads (neighbour index, or three_nn distances and indices) while the current unit's layers
// run: fetch_meta only loads, commit_meta computes and writes the slot tables into LDS.
struct MetaPf {
  int i0, i1, i2;
  float d0, d1, d2;
};

template <int SRC, int P>
PN2_DEV MetaPf fetch_meta(const Params& prm, int tile, int pass, int p) {
  MetaPf f{-1, 0, 0, 0.f, 0.f, 0.f};
  if (SRC == kSrcGroup) {
    const int ns_pad = 1 << prm.lg_ns_pad;
    const int g = prm.passes == 1 ? tile * prm.gpw + (p >> prm.lg_ns_pad) : tile;
    const int k = prm.passes == 1 ? (p & (ns_pad - 1)) : pass * P + p;
    if (g < prm.ngroups) {
      const int kk = k < prm.ns ? k : 0;  // padding slots repeat the first neighbour
      f.i0 = prm.idx[(size_t)g * prm.ns + kk];
    }
  } else if (SRC == kSrcFP) {
    const long long row = (long long)tile * P + p;
    if (row < prm.rows) {
      const float* d = prm.dist + row * 3;
      const int32_t* ii = prm.nn + row * 3;
      f.d0 = d[0];
      f.d1 = d[1];
      f.d2 = d[2];
      f.i0 = ii[0];
      f.i1 = ii[1];
      f.i2 = ii[2];
    }
  }
  return f;
}

template <int SRC, int P>
PN2_DEV void commit_meta(const Params& prm, int tile, int pass, int p, const MetaPf& f,
                         int* s_src, int* s_aux, float* s_pw, float* s_fw, int* s_fi) {
  int src = -1, aux = 0;
  float pw = 0.f;
  if (SRC == kSrcGroup) {
    const int ns_pad = 1 << prm.lg_ns_pad;
    const int g = prm.passes == 1 ? tile * prm.gpw + (p >> prm.lg_ns_pad) : tile;
    const int k = prm.passes == 1 ? (p & (ns_pad - 1)) : pass * P + p;
    if (g < prm.ngroups) {
      const int b = g / prm.M;
      src = b * prm.N + f.i0;
      aux = g;
      if (k < prm.ns) {
        pw = 1.f;
        if (prm.pool == PN2_POOL_WEIGHTED_AVG) {
          // exp(-5 |grouped_xyz|) (pointnet_util.py:136-137)
          const float* q = prm.xyz + (size_t)src * 3;
          const float* c = prm.new_xyz + (size_t)g * 3;
          const float dx = q[0] - c[0], dy = q[1] - c[1], dz = q[2] - c[2];
          pw = expf(-sqrtf((dx * dx + dy * dy) + dz * dz) * 5.0f);
        }
      }
    }
  } else {
    const long long row = (long long)tile * P + p;
    if (row < prm.rows) {
      src = (int)row;
      if (SRC == kSrcFP) {
        const int b = (int)(row / prm.n);
        float w1, w2, w3;
        idw3(f.d0, f.d1, f.d2, w1, w2, w3);
        s_fw[3 * p] = w1;
        s_fw[3 * p + 1] = w2;
        s_fw[3 * p + 2] = w3;
        s_fi[3 * p] = b * prm.m + f.i0;
        s_fi[3 * p + 1] = b * prm.m + f.i1;
        s_fi[3 * p + 2] = b * prm.m + f.i2;
      }
    }
  }
  s_src[p] = src;
  s_aux[p] = aux;
  s_pw[p] = pw;
}

template <int SRC, int R, bool WL>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(2, 2))) void mlp_kernel(const Params prm) {
  constexpr int P = 32 * R;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* act0 = smem;
  float* act1 = smem + prm.off1;
  float* part = smem + prm.off_part;  // pool partials [R][4][2][coutp]
  float* run = smem + prm.off_run;    // running pool over passes [2][coutp]
  int* s_src = reinterpret_cast<int*>(smem + prm.off_meta);  // [P] source row (or -1)
  int* s_aux = s_src + P;                                      // [P] group centre / base row
  float* s_pw = reinterpret_cast<float*>(s_aux + P);           // [P] pool weight per slot
  float* s_fw = s_pw + P;                                      // [P*3] IDW weights (fp source)
  int* s_fi = reinterpret_cast<int*>(s_fw + 3 * P);            // [P*3] neighbour rows
  float* s_norm = reinterpret_cast<float*>(s_fi + 3 * P);      // [kMaxGroupsPerWG]

  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int wave = tid / kWave;
  const int col = lane & 31;
  const int h = lane >> 5;
  const int ns_pad = 1 << prm.lg_ns_pad;
  const bool pooled = (SRC == kSrcGroup) && prm.pool >= 0;
  const LayerDev& LL = prm.L[prm.nl - 1];
  const int coutp = LL.cout32 * 32;
  const float* wl = WL ? smem + prm.off_w : nullptr;
  Ctx ctx{&prm, wl, act0, act1, part, s_src, s_aux, s_pw, lane, col, h, ns_pad, coutp,
          pooled, 0};
  if (WL) {
    // every layer's packed block into LDS once; the loads overlap the metadata phase and
    // the first barrier publishes them
    const float4* src0 = reinterpret_cast<const float4*>(prm.L[0].w);
    (void)src0;
    for (int l = 0; l < prm.nl; ++l) {
      const LayerDev& Ld = prm.L[l];
      const int n4 = (Ld.cout32 * Ld.cin8 * 256 + Ld.cout32 * 64) / 4;
      const float4* src = Ld.w;
      float4* dst = reinterpret_cast<float4*>(smem + prm.off_w + Ld.lofs);
      for (int i0 = tid; i0 < n4; i0 += kBlock * 4) {
        float4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = src[min(i0 + u * kBlock, n4 - 1)];  // branch-free
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (i0 + u * kBlock < n4) dst[i0 + u * kBlock] = v[u];
      }
    }
  }

  // Tiles of this workgroup: prm.tpw consecutive tiles (adjacent groups share cached
  // points; weights staged in LDS are loaded once for all of them).
  const int t_begin = (int)blockIdx.x * prm.tpw;
  const int t_end = min(t_begin + prm.tpw, prm.ntiles);
  // metadata of the first unit; later units' loads are issued one unit ahead (below)
  MetaPf pf{};
  if (t_begin < t_end && tid < P) pf = fetch_meta<SRC, P>(prm, t_begin, 0, tid);

  PN2_STAMP(0);
  for (int tile = t_begin; tile < t_end; ++tile)
  for (int pass = 0; pass < prm.passes; ++pass) {
    ctx.tile = tile;
    // ---- 1. per-slot metadata -----------------------------------------------------------
    if (tid < P) commit_meta<SRC, P>(prm, tile, pass, tid, pf, s_src, s_aux, s_pw, s_fw, s_fi);
    if (pooled && prm.pool == PN2_POOL_WEIGHTED_AVG && pass == 0) {
      // normaliser sum(exp(-5|grouped_xyz|)) over the group's ns entries (:138-139)
      if (prm.passes == 1) {
        __syncthreads();
        for (int gi = wave; gi < prm.gpw; gi += kWaves) {
          float v = 0.f;
          for (int k = lane; k < ns_pad; k += kWave) v += s_pw[(gi << prm.lg_ns_pad) + k];
          v = seg_sum<kWave>(v);
          if (lane == 0) s_norm[gi] = v;
        }
      } else {
        const int g = tile;
        const int b = g / prm.M;
        const float* c = prm.new_xyz + (size_t)g * 3;
        float v = 0.f;
        for (int k = tid; k < prm.ns; k += kBlock) {
          const float* q = prm.xyz + ((size_t)b * prm.N + prm.idx[(size_t)g * prm.ns + k]) * 3;
          const float dx = q[0] - c[0], dy = q[1] - c[1], dz = q[2] - c[2];
          v += expf(-sqrtf((dx * dx + dy * dy) + dz * dz) * 5.0f);
        }
        v = seg_sum<kWave>(v);
        if (lane == 0) s_norm[8 + wave] = v;
        __syncthreads();
        if (tid == 0) s_norm[0] = (s_norm[8] + s_norm[9]) + (s_norm[10] + s_norm[11]);
      }
    }
    __syncthreads();
    if (pooled && prm.pool == PN2_POOL_WEIGHTED_AVG && tid < P) {
      const int gi = prm.passes == 1 ? (tid >> prm.lg_ns_pad) : 0;
      s_pw[tid] = s_pw[tid] / s_norm[gi];
    }

    // ---- 2. gather the input rows into act0 [P][width0] ---------------------------------
    PN2_STAMP(1);
    gather_rows<SRC, P>(prm, act0, s_src, s_aux, s_fw, s_fi);
    __syncthreads();
    PN2_STAMP(2);
    // the next unit's metadata loads, in flight while this unit's layers run
    {
      const bool more_passes = pass + 1 < prm.passes;
      const int nt = more_passes ? tile : tile + 1, np = more_passes ? pass + 1 : 0;
      if (nt < t_end && tid < P) pf = fetch_meta<SRC, P>(prm, nt, np, tid);
    }

    // ---- 3. the layers ------------------------------------------------------------------
    // An item = one 32-column output tile over RG of the R row tiles; layers narrower than
    // the 4 waves split the row tiles so every wave works (nsplit row groups).
    for (int l = 0; l < prm.nl; ++l) {
      const LayerDev& Ld = prm.L[l];
      const bool last = l == prm.nl - 1 && !prm.attn && !prm.stage_out;
      const int c32 = Ld.cout32;
      const int nsplit = item_split(R, c32);
      const int rg_tiles = R / nsplit;
      const int nitems = nsplit * c32;
      for (int item = wave; item < nitems; item += kWaves) {
        const int to = item / nsplit;
        const int rt0 = (item - to * nsplit) * rg_tiles;
        if (rg_tiles == 1) layer_item<SRC, R, 1, WL>(ctx, l, last, to, rt0, pass);
        else layer_item<SRC, R, (R >= 2 ? 2 : 1), WL>(ctx, l, last, to, rt0, pass);
      }
      __syncthreads();
      PN2_STAMP(3 + l);
    }

    if constexpr (SRC == kSrcGroup) {
      if (prm.attn) attention_tail<R>(prm, smem, (prm.nl & 1) ? act1 : act0,
                                      (prm.nl & 1) ? prm.stride1 : prm.stride0, tile);
    } else if (prm.stage_out) {
      // the tile's output rows are contiguous in HBM: one wave per row, whole rows stored
      // coalesced (the next tile's gather writes LDS only after the metadata barrier)
      const int ll = prm.nl - 1;
      const float* src = (ll & 1) ? act0 : act1;
      const int S = (ll & 1) ? prm.stride0 : prm.stride1;
      const int cout = prm.L[ll].cout;
      const long long row0 = (long long)tile * P;
      const int nrows = (int)min((long long)P, prm.rows - row0);
      float* dst = prm.out + row0 * cout;
      if (prm.out_vec) {
        const int c4 = cout >> 2;
        for (int p = wave; p < nrows; p += kWaves)
          for (int c = lane; c < c4; c += kWave)
            reinterpret_cast<float4*>(dst + (size_t)p * cout)[c] =
                *reinterpret_cast<const float4*>(src + p * S + 4 * c);
      } else {
        for (int p = wave; p < nrows; p += kWaves)
          for (int c = lane; c < cout; c += kWave) dst[(size_t)p * cout + c] = src[p * S + c];
      }
    }

    // ---- 4. pooling: combine the row-tile partials of each group, store -----------------
    if (pooled && !prm.direct_pool) {
      const int cout = LL.cout;
      const bool first = pass == 0, final = pass == prm.passes - 1;
      const int ngr = prm.passes == 1 ? prm.gpw : 1;
      const int lg = prm.lg_ns_pad;
      for (int gi = 0; gi < ngr; ++gi) {
        const int g = prm.passes == 1 ? tile * prm.gpw + gi : tile;
        if (g >= prm.ngroups) break;
        int rt0, nrt, u;
        if (prm.passes > 1) { rt0 = 0; nrt = R; u = 0; }
        else if (lg >= 5) { nrt = ns_pad >> 5; rt0 = gi * nrt; u = 0; }
        else { const int gpt = 32 >> lg; rt0 = gi / gpt; nrt = 1; u = gi - rt0 * gpt; }
        for (int fo = tid; fo < cout; fo += kBlock) {
          float mx = -__builtin_inff(), sm = 0.f;
          for (int rt = rt0; rt < rt0 + nrt; ++rt) {
            const float* pp = part + ((size_t)(rt * 4 + u) * 2) * coutp + fo;
            mx = fmaxf(mx, pp[0]);
            sm = sm + pp[coutp];
          }
          if (prm.passes > 1) {
            if (!first) { mx = fmaxf(mx, run[fo]); sm = run[coutp + fo] + sm; }
            run[fo] = mx;
            run[coutp + fo] = sm;
          }
          if (final) store_pooled(prm, g, fo, cout, mx, sm);
        }
      }
      __syncthreads();
    }
  }
  PN2_STAMP(15);
}

// Packed layer: Wp [cout32][cin8][2][32][4] then scale [cout32*32] then shift [cout32*32].
// scale = bn_scale (1 without BN), shift = bias*scale + bn_shift; padded rows/columns are 0.
__global__ void mlp_pack_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                const float* __restrict__ bn_scale,
                                const float* __restrict__ bn_shift, int cin, int cout, int cin8,
                                int cout32, float* __restrict__ packed) {
  const long long nw = (long long)cout32 * cin8 * 256;
  const long long total = nw + 2LL * cout32 * 32;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (e < nw) {
      const int s = (int)(e & 3);
      const int i = (int)((e >> 2) & 31);
      const int hh = (int)((e >> 7) & 1);
      const long long tc = e >> 8;
      const int c = (int)(tc % cin8);
      const int to = (int)(tc / cin8);
      const int f = 8 * c + 4 * hh + s, o = 32 * to + i;
      if (f < cin && o < cout) v = W[(size_t)f * cout + o];
    } else {
      const long long r = e - nw;
      const int which = (int)(r / (cout32 * 32));
      const int o = (int)(r % (cout32 * 32));
      if (o < cout) {
        const float sc = bn_scale ? bn_scale[o] : 1.f;
        if (which == 0) v = sc;
        else v = (bias ? bias[o] : 0.f) * sc + (bn_shift ? bn_shift[o] : 0.f);
      }
    }
    packed[e] = v;
  }
}

int next_pow2(int v) {
  int p = 1;
  while (p < v) p <<= 1;
  return p;
}
int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

constexpr size_t kLdsLimit = 160 * 1024;

// Fill the layer table and LDS layout for R row tiles; returns LDS bytes (0 = invalid).
size_t plan(Params& prm, int nl, const pn2_mlp_layer* layers, int cin0, int R, bool pooled,
            bool wl = false) {
  const int P = 32 * R;
  int wfloats = 0;
  int w0 = ((cin0 + 7) / 8) * 8, w1 = 0;
  for (int l = 0; l < nl; ++l) {
    const pn2_mlp_layer& L = layers[l];
    const int cin8 = (L.cin + 7) / 8, cout32 = (L.cout + 31) / 32;
    const float* base = static_cast<const float*>(L.packed);
    prm.L[l].w = reinterpret_cast<const float4*>(base);
    prm.L[l].scale = base + (size_t)cout32 * cin8 * 256;
    prm.L[l].shift = prm.L[l].scale + cout32 * 32;
    prm.L[l].cin8 = cin8;
    prm.L[l].cout32 = cout32;
    prm.L[l].cout = L.cout;
    prm.L[l].relu = (L.flags & PN2_MLP_RELU) ? 1 : 0;
    prm.L[l].lofs = wfloats;
    wfloats += cout32 * cin8 * 256 + cout32 * 64;
    if (l < nl - 1 || prm.attn || prm.stage_out) {  // layer l writes buffer (l+1)&1
      if ((l + 1) & 1) w1 = w1 > cout32 * 32 ? w1 : cout32 * 32;
      else w0 = w0 > cout32 * 32 ? w0 : cout32 * 32;
    }
  }
  prm.nl = nl;
  prm.width0 = ((cin0 + 7) / 8) * 8;
  // row strides = 4 (mod 32) floats: the 16-byte reads/writes of 8 consecutive rows hit
  // distinct bank quads
  prm.stride0 = ((w0 + 31) / 32) * 32 + 4;
  prm.stride1 = ((w1 + 31) / 32) * 32 + 4;
  const int coutp = prm.L[nl - 1].cout32 * 32;
  size_t off = (size_t)P * prm.stride0;
  prm.off1 = (int)off;
  off += (size_t)P * (w1 ? prm.stride1 : 0);
  prm.off_part = (int)off;
  if (pooled) off += (size_t)R * 4 * 2 * coutp;
  prm.off_run = (int)off;
  if (pooled) off += 2 * (size_t)coutp;
  prm.off_meta = (int)off;
  off += (size_t)P * 9 + kMaxGroupsPerWG;
  off = (off + 3) & ~(size_t)3;
  if (prm.attn) {  // K and V column segments (P rows), queries (one row per group)
    prm.stride_kv = prm.att_wseg + 4;
    prm.stride_q = coutp + 4;
    prm.off_k = (int)off;
    off += (size_t)P * prm.stride_kv;
    prm.off_v = (int)off;
    off += (size_t)P * prm.stride_kv;
    prm.off_q = (int)off;
    off += (size_t)(P >> prm.lg_ns_pad > 0 ? P >> prm.lg_ns_pad : 1) * prm.stride_q;
  }
  prm.off_w = (int)off;
  prm.wfloats = wl ? wfloats : 0;
  off += prm.wfloats;
  return off * sizeof(float);
}

// Input segments of the three sources (see Params).
void set_segments(Params& prm, int nA, bool vecA, int offA, int nB, bool vecB, int offB,
                  int cin_total) {
  prm.vecA = vecA;
  prm.nA = vecA ? nA / 4 : nA;
  prm.offA = offA;
  prm.vecB = vecB;
  prm.nB = vecB ? nB / 4 : nB;
  prm.offB = offB;
  prm.divA = make_fastdiv((uint32_t)(prm.nA > 0 ? prm.nA : 1));
  prm.divB = make_fastdiv((uint32_t)(prm.nB > 0 ? prm.nB : 1));
  prm.cin_total = cin_total;
  const int npad = prm.width0 - cin_total;
  prm.div_pad = make_fastdiv((uint32_t)(npad > 0 ? npad : 1));
}

int check_layers(int nl, const pn2_mlp_layer* layers, int cin0) {
  if (nl < 1 || nl > PN2_MLP_MAX_LAYERS || !layers) return PN2_EINVAL;
  int cin = cin0;
  for (int l = 0; l < nl; ++l) {
    if (!layers[l].packed || layers[l].cin != cin || layers[l].cout <= 0) return PN2_EINVAL;
    if ((reinterpret_cast<uintptr_t>(layers[l].packed) & 15) != 0) return PN2_EINVAL;
    cin = layers[l].cout;
  }
  return PN2_OK;
}

// Compute units of the current device (cached per device id).
int device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 0;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    cache[dev] = n;
  }
  return cache[dev];
}

// Dynamic LDS beyond the 64 KiB default is opted into once per instantiation.
template <int SRC, int R, bool WL>
int launch_one(Params prm, long long nblocks, size_t lds, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void*>(&mlp_kernel<SRC, R, WL>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (int)kLdsLimit);
  if (attr != hipSuccess) return (int)attr;
  prm.ntiles = (int)nblocks;
  // Several consecutive tiles per workgroup (weights staged once, the next tile's metadata
  // loads overlapping the current tile's layers), but only as many as keep >= 4 rounds of
  // workgroups: the dispatcher then still balances around CUs that other streams' kernels
  // hold (a grid of exactly the co-resident slots with static tile ranges waited for the SA1
  // sampler's CUs in the whole-model pipeline).
  prm.tpw = 1;
  constexpr int max_tpw = 8, rounds = 4;  // measured: scripts/ab_tpw.sh
  const long long slots = (long long)device_cus() * (lds * 2 <= kLdsLimit ? 2 : 1);
  while (slots > 0 && prm.tpw * 2 <= max_tpw && nblocks >= slots * rounds * prm.tpw * 2)
    prm.tpw *= 2;
  long long grid = (nblocks + prm.tpw - 1) / prm.tpw;
#ifdef PN2_MLP_STAMP
  prm.stamp = g_stamp;
  prm.tpw = 1;  // one tile per workgroup: the stamps are per tile
  grid = nblocks;
#endif
  hipLaunchKernelGGL((mlp_kernel<SRC, R, WL>), dim3((unsigned)grid), dim3(kBlock), lds, s, prm);
  PN2_RETURN_LAUNCH();
}

template <int SRC>
int launch_rows_R(Params& prm, int R, long long nblocks, size_t lds, hipStream_t s) {
  if (nblocks <= 0) return PN2_OK;
  if (nblocks > 0x7fffffffLL) return PN2_EINVAL;
  if (prm.wfloats) {  // weights staged in LDS (small MLPs of the SA layers)
    if (SRC != kSrcGroup) return PN2_EINVAL;
    if (R == 1) return launch_one<kSrcGroup, 1, true>(prm, nblocks, lds, s);
    if (R == 2) return launch_one<kSrcGroup, 2, true>(prm, nblocks, lds, s);
    return launch_one<kSrcGroup, 4, true>(prm, nblocks, lds, s);
  }
  if (R == 1) return launch_one<SRC, 1, false>(prm, nblocks, lds, s);
  if (R == 2) return launch_one<SRC, 2, false>(prm, nblocks, lds, s);
  return launch_one<SRC, 4, false>(prm, nblocks, lds, s);
}

// Row tiles per workgroup: prefer the cheapest R whose LDS lets two
// workgroups share a CU (one wave per SIMD leaves every stall exposed), then any that fits.
int choose_R(Params& prm, int nl, const pn2_mlp_layer* layers, int cin0, bool pooled,
             long long tiles32, int min_R, size_t* lds_out) {
  int best = 0, best_occ = 0;
  double best_cost = 0;
  size_t best_lds = 0;
  for (int R = 4; R >= min_R; R >>= 1) {
    const size_t lds = plan(prm, nl, layers, cin0, R, pooled);
    if (lds > kLdsLimit) continue;
    if (R > 1 && tiles32 < 256LL * R) continue;  // too few workgroups to fill the chip
    // per row tile: items per wave x (RG row tiles x cin8 chunks + ~4 chunks of exposed
    // weight-load latency per item), the kernel's item split (see mlp_kernel, section 3)
    double cost = 0;
    for (int l = 0; l < nl; ++l) {
      const int c32 = (layers[l].cout + 31) / 32, cin8 = (layers[l].cin + 7) / 8;
      const int nsplit = item_split(R, c32);
      const int items = nsplit * c32, rg = R / nsplit;
      cost += (double)((items + kWaves - 1) / kWaves) * (rg * cin8 + 4) / R;
    }
    const int occ = lds * 2 <= kLdsLimit ? 2 : 1;
    if (!best || occ > best_occ || (occ == best_occ && cost < best_cost)) {
      best = R;
      best_occ = occ;
      best_cost = cost;
      best_lds = lds;
    }
  }
  if (best) {
    *lds_out = plan(prm, nl, layers, cin0, best, pooled);
    (void)best_lds;
  }
  return best;
}

// Per-point outputs (fp / rows sources): stage the last layer through LDS when that fits the
// same occupancy, else store it from the registers.
int choose_R_staged(Params& prm, int nl, const pn2_mlp_layer* layers, int cin0, long long tiles32,
                    const float* out, size_t* lds_out) {
  Params plain = prm;
  size_t lds_plain = 0;
  const int R_plain = choose_R(plain, nl, layers, cin0, false, tiles32, 1, &lds_plain);
  {
    Params staged = prm;
    staged.stage_out = 1;
    size_t lds = 0;
    const int R = choose_R(staged, nl, layers, cin0, false, tiles32, 1, &lds);
    const int occ = lds * 2 <= kLdsLimit ? 2 : 1, occ_plain = lds_plain * 2 <= kLdsLimit ? 2 : 1;
    if (R && (!R_plain || (R == R_plain && occ == occ_plain))) {
      const int cout = layers[nl - 1].cout;
      staged.out_vec = (cout % 4 == 0) && ((reinterpret_cast<uintptr_t>(out) & 15) == 0);
      prm = staged;
      *lds_out = lds;
      return R;
    }
  }
  prm = plain;
  *lds_out = lds_plain;
  return R_plain;
}

}  // namespace
}  // namespace pn2

extern "C" {

#ifdef PN2_MLP_STAMP
// diagnostic builds only (tools/stamp_mlp.py): device buffer of kStampWG x 16 u64, or NULL
void pn2_mlp_set_stamp(void* buf) { pn2::g_stamp = static_cast<unsigned long long*>(buf); }
#endif

size_t pn2_mlp_packed_size(int cin, int cout) {
  if (cin <= 0 || cout <= 0) return 0;
  const size_t cin8 = (size_t)(cin + 7) / 8, cout32 = (size_t)(cout + 31) / 32;
  return (cout32 * cin8 * 256 + 2 * cout32 * 32) * sizeof(float);
}

int pn2_mlp_pack(const float* weight, const float* bias, const float* bn_scale,
                 const float* bn_shift, int cin, int cout, void* packed, size_t packed_bytes,
                 pn2_stream_t stream) {
  if (cin <= 0 || cout <= 0 || !weight || !packed) return PN2_EINVAL;
  if (packed_bytes < pn2_mlp_packed_size(cin, cout)) return PN2_EINVAL;
  if ((!bn_scale) != (!bn_shift)) return PN2_EINVAL;
  if ((reinterpret_cast<uintptr_t>(packed) & 15) != 0) return PN2_EINVAL;
  const int cin8 = (cin + 7) / 8, cout32 = (cout + 31) / 32;
  const long long total = (long long)cout32 * cin8 * 256 + 2LL * cout32 * 32;
  long long blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(pn2::mlp_pack_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, weight, bias, bn_scale, bn_shift, cin, cout, cin8,
                     cout32, static_cast<float*>(packed));
  PN2_RETURN_LAUNCH();
}

static int group_mlp_impl(const float* xyz, const float* points, const float* new_xyz,
                          const int32_t* idx, int B, int N, int C, int M, int nsample, int flags,
                          int nlayers, const pn2_mlp_layer* layers, int pool,
                          const pn2_mlp_layer* qkv, const float* bn_scale, const float* bn_shift,
                          int add_max, float* out, hipStream_t stream) {
  using namespace pn2;
  if (B < 0 || N < 0 || C < 0 || M < 0 || nsample <= 0) return PN2_EINVAL;
  if (pool < PN2_POOL_NONE || pool > PN2_POOL_MAX_AND_AVG) return PN2_EINVAL;
  int layout, cin0;
  if (!points) { layout = kXyzOnly; cin0 = 3; }
  else if (!(flags & PN2_USE_XYZ)) { layout = kPointsOnly; cin0 = C; }
  else { layout = (flags & PN2_XYZ_LAST) ? kXyzLast : kXyzFirst; cin0 = C + 3; }
  int rc = check_layers(nlayers, layers, cin0);
  if (rc) return rc;
  const int ns_pad = nsample < 8 ? 8 : next_pow2(nsample);
  Params prm = {};
  prm.lg_ns_pad = ilog2(ns_pad);
  int min_R = 1;
  if (qkv) {
    const int Ca = layers[nlayers - 1].cout;
    if (Ca % 32 || (!bn_scale) != (!bn_shift)) return PN2_EINVAL;
    for (int i = 0; i < 3; ++i) {
      if (!qkv[i].packed || qkv[i].cin != Ca || qkv[i].cout != Ca || (qkv[i].flags & PN2_MLP_RELU))
        return PN2_EINVAL;
      if ((reinterpret_cast<uintptr_t>(qkv[i].packed) & 15) != 0) return PN2_EINVAL;
    }
    if (ns_pad > 128) return PN2_EINVAL;  // one pass: the group's rows all in one workgroup
    prm.attn = 1;
    // column segments of K and V: whole rows when a head spans rows (C <= 4 ns), else blocks
    // of 4 ns columns (each completes the heads of its column block)
    prm.att_wseg = (Ca <= 4 * nsample || Ca % (4 * nsample) || (4 * nsample) % 32) ? Ca
                                                                                    : 4 * nsample;
    prm.att_nseg = Ca / prm.att_wseg;
    prm.att_add_max = add_max ? 1 : 0;
    prm.att_scale = bn_scale;
    prm.att_shift = bn_shift;
    pool = PN2_POOL_NONE;
    min_R = ns_pad > 32 ? ns_pad / 32 : 1;
  }
  const long long ngroups = (long long)B * M;
  if (ngroups == 0) return PN2_OK;
  if (!xyz || !new_xyz || !idx || !out || ngroups > 0x7fffffffLL) return PN2_EINVAL;
  if ((long long)B * N > 0x7fffffffLL || ngroups * nsample > 0x7fffffffLL) return PN2_EINVAL;
  const bool pooled = pool >= 0;
  size_t lds = 0;
  // a single-pass workgroup holds whole groups: P = 32R must be a multiple of ns_pad, or
  // the group is processed in ns_pad / P passes of one workgroup
  const long long tiles32 = (ngroups * ns_pad + 31) / 32;
  const int R = choose_R(prm, nlayers, layers, cin0, pooled, tiles32, min_R, &lds);
  if (!R) return PN2_EINVAL;
  const int P = 32 * R;
  if (qkv) {
    for (int i = 0; i < 3; ++i) {
      const int cin8 = (qkv[i].cin + 7) / 8, cout32 = qkv[i].cout / 32;
      const float* base = static_cast<const float*>(qkv[i].packed);
      prm.qkv[i].w = reinterpret_cast<const float4*>(base);
      prm.qkv[i].scale = base + (size_t)cout32 * cin8 * 256;
      prm.qkv[i].shift = prm.qkv[i].scale + cout32 * 32;
      prm.qkv[i].cin8 = cin8;
      prm.qkv[i].cout32 = cout32;
      prm.qkv[i].cout = qkv[i].cout;
      prm.qkv[i].relu = 0;
    }
  }
  prm.xyz = xyz;
  prm.points = points;
  prm.new_xyz = new_xyz;
  prm.idx = idx;
  prm.N = N;
  prm.C = C;
  prm.M = M;
  prm.ns = nsample;
  prm.layout = layout;
  if (layout == kXyzOnly) set_segments(prm, 0, false, 0, 3, false, 0, 3);
  else if (layout == kPointsOnly) set_segments(prm, C, C % 4 == 0, 0, 0, false, 0, C);
  else if (layout == kXyzFirst) set_segments(prm, C, C % 4 == 0, 3, 3, false, 0, C + 3);
  else set_segments(prm, C, C % 4 == 0, 0, 3, false, C, C + 3);
  prm.ngroups = (int)ngroups;
  prm.pool = pool;
  prm.out = out;
  long long nblocks;
  if (ns_pad <= P) {
    prm.passes = 1;
    prm.gpw = P / ns_pad;
    nblocks = (ngroups + prm.gpw - 1) / prm.gpw;
  } else {
    prm.passes = ns_pad / P;
    prm.gpw = 1;
    nblocks = ngroups;
  }
  if (pooled && prm.gpw > kMaxGroupsPerWG) return PN2_EINVAL;
  prm.direct_pool = pooled && prm.passes == 1 && ns_pad <= 32;
  {
    // small MLPs: stage every layer's weights in LDS when two workgroups still fit a CU
    Params p2 = prm;
    const size_t lds_wl = plan(p2, nlayers, layers, cin0, R, pooled, true);
    if (lds_wl * 2 <= kLdsLimit) {
      prm = p2;
      lds = lds_wl;
    }
  }
  return launch_rows_R<kSrcGroup>(prm, R, nblocks, lds, stream);
}

int pn2_group_mlp(const float* xyz, const float* points, const float* new_xyz,
                  const int32_t* idx, int B, int N, int C, int M, int nsample, int flags,
                  int nlayers, const pn2_mlp_layer* layers, int pool, float* out,
                  pn2_stream_t stream) {
  return group_mlp_impl(xyz, points, new_xyz, idx, B, N, C, M, nsample, flags, nlayers, layers,
                        pool, nullptr, nullptr, nullptr, 0, out, (hipStream_t)stream);
}

int pn2_group_mlp_attention(const float* xyz, const float* points, const float* new_xyz,
                            const int32_t* idx, int B, int N, int C, int M, int nsample,
                            int flags, int nlayers, const pn2_mlp_layer* layers,
                            const pn2_mlp_layer* qkv, const float* bn_scale,
                            const float* bn_shift, int add_max, float* out,
                            pn2_stream_t stream) {
  if (!qkv) return PN2_EINVAL;
  return group_mlp_impl(xyz, points, new_xyz, idx, B, N, C, M, nsample, flags, nlayers, layers,
                        PN2_POOL_NONE, qkv, bn_scale, bn_shift, add_max, out,
                        (hipStream_t)stream);
}

int pn2_fp_mlp(const float* dist, const int32_t* nn_idx, const float* points1, int C1,
               const float* points2, int C2, int B, int n, int m, int nlayers,
               const pn2_mlp_layer* layers, float* out, pn2_stream_t stream) {
  using namespace pn2;
  if (B < 0 || n < 0 || m < 0 || C1 < 0 || C2 <= 0) return PN2_EINVAL;
  if (C1 > 0 && !points1) return PN2_EINVAL;
  int rc = check_layers(nlayers, layers, C1 + C2);
  if (rc) return rc;
  const long long rows = (long long)B * n;
  if (rows == 0) return PN2_OK;
  if (!dist || !nn_idx || !points2 || !out || m < 1) return PN2_EINVAL;
  if (rows > 0x7fffffffLL || (long long)B * m > 0x7fffffffLL) return PN2_EINVAL;
  Params prm = {};
  size_t lds = 0;
  const int R = choose_R_staged(prm, nlayers, layers, C1 + C2, (rows + 31) / 32, out, &lds);
  if (!R) return PN2_EINVAL;
  prm.dist = dist;
  prm.nn = nn_idx;
  prm.p1 = points1;
  prm.p2 = points2;
  prm.C1 = C1;
  prm.C2 = C2;
  prm.n = n;
  prm.m = m;
  prm.rows = rows;
  set_segments(prm, C2, C2 % 4 == 0, 0, C1, C1 % 4 == 0 && C2 % 4 == 0, C2, C1 + C2);
  prm.passes = 1;
  prm.pool = PN2_POOL_NONE;
  prm.out = out;
  const long long nblocks = (rows + 32 * R - 1) / (32 * R);
  return launch_rows_R<kSrcFP>(prm, R, nblocks, lds, (hipStream_t)stream);
}

int pn2_shared_mlp(const float* x, long long rows, int cin, int nlayers,
                   const pn2_mlp_layer* layers, float* out, pn2_stream_t stream) {
  using namespace pn2;
  if (rows < 0 || cin <= 0) return PN2_EINVAL;
  int rc = check_layers(nlayers, layers, cin);
  if (rc) return rc;
  if (rows == 0) return PN2_OK;
  if (!x || !out || rows > 0x7fffffffLL) return PN2_EINVAL;
  Params prm = {};
  size_t lds = 0;
  const int R = choose_R_staged(prm, nlayers, layers, cin, (rows + 31) / 32, out, &lds);
  if (!R) return PN2_EINVAL;
  prm.x = x;
  prm.cin = cin;
  prm.rows = rows;
  set_segments(prm, cin, cin % 4 == 0, 0, 0, false, 0, cin);
  prm.passes = 1;
  prm.pool = PN2_POOL_NONE;
  prm.out = out;
  const long long nblocks = (rows + 32 * R - 1) / (32 * R);
  return launch_rows_R<kSrcRows>(prm, R, nblocks, lds, (hipStream_t)stream);
}

}  // extern "C"
