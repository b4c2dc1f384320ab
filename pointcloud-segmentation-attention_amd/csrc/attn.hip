// Per-group attention reduction and SA pooling for gfx950.
//
// Replaces the reduction core of AttentionLayer.call
// (attention_points/attention_scannet/attention_layer.py:35-42; instantiated with
// key_dim = output_dim = 4, num_heads = C/4 at :256-258 and :313-315) — six TF ops per SA
// layer (reshape, matmul, div, softmax, matmul, reshape) on 1x4 by 4xns heads — and the
// pooling variants of pointnet_util.py:130-145 (max / avg / weighted_avg / max_and_avg).
//
// The reshape quirk is reproduced, not fixed: tf.reshape of K and V from (B,M,ns,4H) to
// (B,M,H,ns,4) is a row-major reinterpretation, so head h reads the CONTIGUOUS block
// [4*ns*h, 4*ns*(h+1)) of the group's flattened ns*C values as ns pseudo-keys of width 4.
// That makes every head a 16*ns-byte contiguous slab: a lane loads one pseudo-key as one
// float4 (ns lanes per head, 64/ns heads per wave instruction = 1 KiB fully coalesced), the
// softmax max/sum and the four weighted sums are lane-segment reductions in registers, and
// one lane per head stores the head's 4 outputs as one float4. K and V are read exactly once.
#include <math.h>

#include "common.h"

namespace pn2 {
namespace {

constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
// tasks in flight per wave; blocks per CU before the grid strides (8 x 4 waves = a full CU);
// K / V loaded non-temporal (streamed once). The four SSG layers in one launch, no data reused
// from the last-level cache (tools/bench_attn.py `layers4`, profiles/r5/attn*): 117 us with
// 16 blocks per CU and plain loads, 107 non-temporal, 99.7 non-temporal at 8 blocks per CU
// (5.2 TB/s); 4 tasks in flight or 1, and 4 or 32 blocks per CU, were slower
constexpr int kAttnTif = 2;
constexpr int kAttnBlocksPerCu = 8;
// K / V are streamed once: non-temporal loads (no reuse in the caches)
PN2_DEV float4 ld_stream(const float* p) {
  using v4 = float __attribute__((ext_vector_type(4)));
  const v4 r = __builtin_nontemporal_load(reinterpret_cast<const v4*>(p));
  return make_float4(r.x, r.y, r.z, r.w);
}

PN2_DEV float dot4(float4 q, float4 k) {  // (1x4)·(4x1) of tf.matmul, summed left to right
  float s = q.x * k.x;
  s = s + q.y * k.y;
  s = s + q.z * k.z;
  s = s + q.w * k.w;
  return s;
}

// Segment reductions over LPH = 8..64 lanes with DPP / permlane exchanges (no LDS crossbar
// round trip per step, unlike ds_bpermute shuffles): quad xor1 / xor2, row_half_mirror,
// row_mirror, then the gfx950 row swaps. Every lane of a segment ends with the same value.
template <int CTRL>
PN2_DEV float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int SEG, bool MAX>
PN2_DEV float seg_reduce(float v) {
  auto op = [](float a, float b) { return MAX ? fmaxf(a, b) : a + b; };
  v = op(v, dppf<kDppXor1>(v));
  v = op(v, dppf<kDppXor2>(v));
  if constexpr (SEG >= 8) v = op(v, dppf<kDppHalfMirror>(v));
  if constexpr (SEG >= 16) v = op(v, dppf<kDppMirror>(v));
  if constexpr (SEG >= 32) {
    const int u = __float_as_int(v);
    auto x = __builtin_amdgcn_permlane16_swap(u, u, false, false);
    v = op(__int_as_float((int)x[0]), __int_as_float((int)x[1]));
  }
  if constexpr (SEG >= 64) {
    const int u = __float_as_int(v);
    auto x = __builtin_amdgcn_permlane32_swap(u, u, false, false);
    v = op(__int_as_float((int)x[0]), __int_as_float((int)x[1]));
  }
  return v;
}

// One attention reduction: G groups of ns = NS pseudo-keys, C channels, `steps` wave tasks
// (head groups) per group.
struct AttnLayer {
  const float* Q;
  const float* K;
  const float* V;
  float* out;
  int G, C, steps;
  FastDiv div_steps;
};

// NS = nsample (power of two). LPH lanes per head, KPL pseudo-keys per lane, HPW heads per
// wave task; a wave keeps TIF tasks in flight (their K / V loads issued before any reduction).
// Several layers of the same nsample in one launch (the SSG stack's four attention
// reductions): one task space, layer li's tasks at [first[li], first[li + 1]).
constexpr int kAttnMaxLayers = PN2_ATTN_MAX_LAYERS;
struct AttnLayers {
  AttnLayer l[kAttnMaxLayers];
  long long first[kAttnMaxLayers + 1];
  int nlayers;
};

template <int NS, int TIF>
__global__ __launch_bounds__(kBlock) void attn_reduce_kernel(AttnLayers A) {
  constexpr int LPH = NS < kWave ? NS : kWave;
  constexpr int KPL = NS / LPH;
  constexpr int HPW = kWave / LPH;  // heads per wave step
  const int lane = lane_id();
  const int hl = lane / LPH, sl = lane % LPH;
  const long long tasks = A.first[A.nlayers];
  const long long nwaves = (long long)gridDim.x * kWavesPerBlock;
  for (long long t0 = (long long)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; t0 < tasks;
       t0 += nwaves * TIF) {
    float4 q[TIF], k[TIF][KPL], v[TIF][KPL];
    float* op[TIF];
    bool ok[TIF];
#pragma unroll
    for (int i = 0; i < TIF; ++i) {
      long long task = t0 + i * nwaves;
      ok[i] = task < tasks;
      task = ok[i] ? task : t0;
      int li = 0;  // (wave-uniform)
      while (li + 1 < A.nlayers && task >= A.first[li + 1]) ++li;
      const AttnLayer& L = A.l[li];
      const uint32_t lt = (uint32_t)(task - A.first[li]);
      const uint32_t g = fdiv(lt, L.div_steps);
      const int step = (int)(lt - g * (uint32_t)L.steps);
      const int H = L.C / 4;
      const int h = step * HPW + hl;
      ok[i] = ok[i] && h < H;
      const int hh = h < H ? h : 0;
      q[i] = *reinterpret_cast<const float4*>(L.Q + (size_t)g * L.C + 4 * hh);
      const float* Kh = L.K + (size_t)g * NS * L.C + (size_t)hh * 4 * NS;  // reshape quirk (:35-36)
      const float* Vh = L.V + (size_t)g * NS * L.C + (size_t)hh * 4 * NS;
#pragma unroll
      for (int kk = 0; kk < KPL; ++kk) {
        const int s = sl + kk * LPH;
        k[i][kk] = ld_stream(Kh + 4 * s);
        v[i][kk] = ld_stream(Vh + 4 * s);
      }
      op[i] = L.out + (size_t)g * L.C + 4 * h;
    }
#pragma unroll
    for (int i = 0; i < TIF; ++i) {
      float sc[KPL];
      float mx = -__builtin_inff();
#pragma unroll
      for (int kk = 0; kk < KPL; ++kk) {
        sc[kk] = dot4(q[i], k[i][kk]) / 2.0f;  // / tf.sqrt(key_dim = 4)  (:38)
        mx = fmaxf(mx, sc[kk]);
      }
      mx = seg_reduce<LPH, true>(mx);  // softmax over the ns pseudo-keys (:39)
      float sum = 0.0f;
#pragma unroll
      for (int kk = 0; kk < KPL; ++kk) {
        sc[kk] = expf(sc[kk] - mx);
        sum = sum + sc[kk];
      }
      sum = seg_reduce<LPH, false>(sum);
      float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int kk = 0; kk < KPL; ++kk) {
        const float w = sc[kk] / sum;
        o.x = o.x + w * v[i][kk].x;  // aᵀ·V_h (:40)
        o.y = o.y + w * v[i][kk].y;
        o.z = o.z + w * v[i][kk].z;
        o.w = o.w + w * v[i][kk].w;
      }
      o.x = seg_reduce<LPH, false>(o.x);
      o.y = seg_reduce<LPH, false>(o.y);
      o.z = seg_reduce<LPH, false>(o.z);
      o.w = seg_reduce<LPH, false>(o.w);
      if (sl == 0 && ok[i]) *reinterpret_cast<float4*>(op[i]) = o;  // (:42)
    }
  }
}

// Any nsample: one wave per (group, head), lanes stride over the pseudo-keys, running
// (max, sum, weighted sum) per lane merged across the wave.
__global__ __launch_bounds__(kBlock) void attn_reduce_generic_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V, int G,
    int ns, int C, float* __restrict__ out) {
  const int lane = lane_id();
  const int H = C / 4;
  const long long tasks = (long long)G * H;
  const long long nwaves = (long long)gridDim.x * kWavesPerBlock;
  for (long long task = (long long)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; task < tasks;
       task += nwaves) {
    const long long g = task / H;
    const int h = (int)(task - g * H);
    const float4 q = *reinterpret_cast<const float4*>(Q + g * C + 4 * h);
    const float* Kh = K + g * (long long)ns * C + (long long)h * 4 * ns;
    const float* Vh = V + g * (long long)ns * C + (long long)h * 4 * ns;
    float mx = -__builtin_inff();
    for (int s = lane; s < ns; s += kWave)
      mx = fmaxf(mx, dot4(q, *reinterpret_cast<const float4*>(Kh + 4 * s)) / 2.0f);
    mx = seg_max<kWave>(mx);
    float sum = 0.f;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = lane; s < ns; s += kWave) {
      const float e = expf(dot4(q, *reinterpret_cast<const float4*>(Kh + 4 * s)) / 2.0f - mx);
      const float4 v = *reinterpret_cast<const float4*>(Vh + 4 * s);
      sum = sum + e;
      o.x = o.x + e * v.x;
      o.y = o.y + e * v.y;
      o.z = o.z + e * v.z;
      o.w = o.w + e * v.w;
    }
    sum = seg_sum<kWave>(sum);
    o.x = seg_sum<kWave>(o.x) / sum;
    o.y = seg_sum<kWave>(o.y) / sum;
    o.z = seg_sum<kWave>(o.z) / sum;
    o.w = seg_sum<kWave>(o.w) / sum;
    if (lane == 0) *reinterpret_cast<float4*>(out + g * C + 4 * h) = o;
  }
}

// Backward of the reduction (what TF's autodiff of attention_layer.py:35-42 computes), one wave
// per (group, head), lanes striding over the ns pseudo-keys. With s_i = q.K_i / 2,
// a = softmax(s), o = sum_i a_i V_i and the incoming gradient dO (4 floats per head):
//   dV_i = a_i dO,   ds_i = a_i (dO.V_i - dO.o),   dK_i = ds_i q / 2,   dq = sum_i ds_i K_i / 2.
// The forward is recomputed (max, normaliser, o) so nothing is stored between the passes.
__global__ __launch_bounds__(kBlock) void attn_reduce_grad_kernel(
    const float* __restrict__ Q, const float* __restrict__ K, const float* __restrict__ V,
    const float* __restrict__ dO, int G, int ns, int C, float* __restrict__ dQ,
    float* __restrict__ dK, float* __restrict__ dV) {
  const int lane = lane_id();
  const int H = C / 4;
  const long long tasks = (long long)G * H;
  const long long nwaves = (long long)gridDim.x * kWavesPerBlock;
  for (long long task = (long long)blockIdx.x * kWavesPerBlock + threadIdx.x / kWave; task < tasks;
       task += nwaves) {
    const long long g = task / H;
    const int h = (int)(task - g * H);
    const float4 q = *reinterpret_cast<const float4*>(Q + g * C + 4 * h);
    const float4 go = *reinterpret_cast<const float4*>(dO + g * C + 4 * h);
    const size_t off = (size_t)g * ns * C + (size_t)h * 4 * ns;  // reshape quirk (:35-36)
    const float* Kh = K + off;
    const float* Vh = V + off;
    float mx = -__builtin_inff();
    for (int s = lane; s < ns; s += kWave)
      mx = fmaxf(mx, dot4(q, *reinterpret_cast<const float4*>(Kh + 4 * s)) / 2.0f);
    mx = seg_max<kWave>(mx);
    float sum = 0.f;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = lane; s < ns; s += kWave) {
      const float e = expf(dot4(q, *reinterpret_cast<const float4*>(Kh + 4 * s)) / 2.0f - mx);
      const float4 v = *reinterpret_cast<const float4*>(Vh + 4 * s);
      sum = sum + e;
      o.x = o.x + e * v.x;
      o.y = o.y + e * v.y;
      o.z = o.z + e * v.z;
      o.w = o.w + e * v.w;
    }
    sum = seg_sum<kWave>(sum);
    const float inv = 1.0f / sum;
    const float go_o = dot4(go, make_float4(seg_sum<kWave>(o.x) * inv, seg_sum<kWave>(o.y) * inv,
                                            seg_sum<kWave>(o.z) * inv, seg_sum<kWave>(o.w) * inv));
    float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s = lane; s < ns; s += kWave) {
      const float4 k = *reinterpret_cast<const float4*>(Kh + 4 * s);
      const float4 v = *reinterpret_cast<const float4*>(Vh + 4 * s);
      const float a = expf(dot4(q, k) / 2.0f - mx) * inv;
      const float ds = a * (dot4(go, v) - go_o);
      const float hds = ds / 2.0f;
      *reinterpret_cast<float4*>(dV + off + 4 * s) =
          make_float4(a * go.x, a * go.y, a * go.z, a * go.w);
      *reinterpret_cast<float4*>(dK + off + 4 * s) =
          make_float4(hds * q.x, hds * q.y, hds * q.z, hds * q.w);
      gq.x = gq.x + hds * k.x;
      gq.y = gq.y + hds * k.y;
      gq.z = gq.z + hds * k.z;
      gq.w = gq.w + hds * k.w;
    }
    gq.x = seg_sum<kWave>(gq.x);
    gq.y = seg_sum<kWave>(gq.y);
    gq.z = seg_sum<kWave>(gq.z);
    gq.w = seg_sum<kWave>(gq.w);
    if (lane == 0) *reinterpret_cast<float4*>(dQ + g * C + 4 * h) = gq;
  }
}

// One wave per group, lanes over channels (pointnet_util.py:130-145).
__global__ __launch_bounds__(kBlock) void group_pool_kernel(const float* __restrict__ x,
                                                            const float* __restrict__ gxyz, int G,
                                                            int ns, int C, int mode,
                                                            float* __restrict__ out) {
  __shared__ float s_w[kWavesPerBlock][256];
  const int lane = lane_id(), w = threadIdx.x / kWave;
  for (long long g = (long long)blockIdx.x * kWavesPerBlock + w; g < G;
       g += (long long)gridDim.x * kWavesPerBlock) {
    const float* X = x + g * (long long)ns * C;
    if (mode == PN2_POOL_WEIGHTED_AVG) {
      // dists = |grouped_xyz| (:136), exp(-5 d) (:137), normalised over ns (:138-139)
      float part = 0.f;
      for (int k = lane; k < ns; k += kWave) {
        const float* p = gxyz + (g * ns + k) * 3;
        const float d = sqrtf((p[0] * p[0] + p[1] * p[1]) + p[2] * p[2]);
        const float e = expf(-d * 5.0f);
        s_w[w][k] = e;
        part = part + e;
      }
      const float tot = seg_sum<kWave>(part);
      for (int k = lane; k < ns; k += kWave) s_w[w][k] = s_w[w][k] / tot;
    }
    for (int c = lane; c < C; c += kWave) {
      float mx = -__builtin_inff(), sum = 0.f;
      for (int k = 0; k < ns; ++k) {
        const float v = X[(size_t)k * C + c];
        mx = fmaxf(mx, v);
        sum = (mode == PN2_POOL_WEIGHTED_AVG) ? sum + v * s_w[w][k] : sum + v;
      }
      const float avg = sum / (float)ns;
      if (mode == PN2_POOL_MAX) out[g * C + c] = mx;
      else if (mode == PN2_POOL_AVG) out[g * C + c] = avg;
      else if (mode == PN2_POOL_WEIGHTED_AVG) out[g * C + c] = sum;
      else { out[g * 2 * C + c] = avg; out[g * 2 * C + C + c] = mx; }  // [avg, max] (:145)
    }
  }
}

unsigned grid_for(long long waves, int per_cu = 16) {
  long long blocks = (waves + kWavesPerBlock - 1) / kWavesPerBlock;
  if (blocks > 256LL * per_cu) blocks = 256LL * per_cu;  // grid-stride beyond
  return (unsigned)(blocks > 0 ? blocks : 1);
}

// every layer of A shares nsample NS; fills each layer's task stepping and A.first
template <int NS>
void launch_attn(AttnLayers& A, hipStream_t s) {
  constexpr int LPH = NS < kWave ? NS : kWave;
  constexpr int HPW = kWave / LPH;
  long long tasks = 0;
  for (int i = 0; i < A.nlayers; ++i) {
    AttnLayer& L = A.l[i];
    L.steps = (L.C / 4 + HPW - 1) / HPW;
    L.div_steps = make_fastdiv((uint32_t)L.steps);
    A.first[i] = tasks;
    tasks += (long long)L.G * L.steps;
  }
  A.first[A.nlayers] = tasks;
  constexpr int TIF = kAttnTif;
  hipLaunchKernelGGL((attn_reduce_kernel<NS, TIF>),
                     dim3(grid_for((tasks + TIF - 1) / TIF, kAttnBlocksPerCu)),
                     dim3(kBlock), 0, s, A);
}

int attn_launch(AttnLayers& a, int ns, hipStream_t s) {
  if (ns == 8) launch_attn<8>(a, s);
  else if (ns == 16) launch_attn<16>(a, s);
  else if (ns == 32) launch_attn<32>(a, s);
  else if (ns == 64) launch_attn<64>(a, s);
  else if (ns == 128) launch_attn<128>(a, s);
  else return PN2_EINVAL;
  return PN2_OK;
}

// a layer's FastDiv task arithmetic stays exact (worst case HPW = 1)
bool attn_small_tasks(long long G, int C) {
  const long long steps_max = (long long)C / 4;
  return G * steps_max * steps_max < (1LL << 32);
}

}  // namespace
}  // namespace pn2

extern "C" {

int pn2_attn_reduce(const float* Q, const float* K, const float* V, int B, int M, int ns, int C,
                    float* out, pn2_stream_t stream) {
  if (B < 0 || M < 0 || ns <= 0 || C < 0 || (C % 4) != 0) return PN2_EINVAL;
  const long long G = (long long)B * M;
  if (G == 0 || C == 0) return PN2_OK;
  if (!Q || !K || !V || !out || G > INT32_MAX) return PN2_EINVAL;
  if ((((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V | (uintptr_t)out) & 15) != 0) return PN2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  pn2::AttnLayers a{};
  a.l[0] = pn2::AttnLayer{Q, K, V, out, (int)G, C, 0, {}};
  a.nlayers = 1;
  if (!pn2::attn_small_tasks(G, C) || pn2::attn_launch(a, ns, s) != PN2_OK)
    hipLaunchKernelGGL(pn2::attn_reduce_generic_kernel,
                       dim3(pn2::grid_for(G * (C / 4))), dim3(pn2::kBlock), 0, s, Q, K, V,
                       (int)G, ns, C, out);
  PN2_RETURN_LAUNCH();
}

int pn2_attn_reduce_layers(const pn2_attn_layer* layers, int nlayers, int B,
                           pn2_stream_t stream) {
  if (!layers || nlayers < 1 || nlayers > PN2_ATTN_MAX_LAYERS || B < 0) return PN2_EINVAL;
  hipStream_t s = (hipStream_t)stream;
  pn2::AttnLayers a{}, big{};
  int ns = 0;
  for (int i = 0; i < nlayers; ++i) {
    const pn2_attn_layer& l = layers[i];
    if (l.M < 0 || l.ns <= 0 || l.C < 0 || (l.C % 4) != 0) return PN2_EINVAL;
    if (ns && l.ns != ns) return PN2_EINVAL;  // one nsample per launch
    ns = l.ns;
    const long long G = (long long)B * l.M;
    if (G == 0 || l.C == 0) continue;
    if (!l.Q || !l.K || !l.V || !l.out || G > INT32_MAX) return PN2_EINVAL;
    if ((((uintptr_t)l.Q | (uintptr_t)l.K | (uintptr_t)l.V | (uintptr_t)l.out) & 15) != 0)
      return PN2_EINVAL;
    // a layer too large for the FastDiv task arithmetic: its own generic launch, as
    // pn2_attn_reduce runs it (the same results)
    pn2::AttnLayers& dst = pn2::attn_small_tasks(G, l.C) ? a : big;
    dst.l[dst.nlayers++] = pn2::AttnLayer{l.Q, l.K, l.V, l.out, (int)G, l.C, 0, {}};
  }
  // an nsample the layers kernel has no instance for: every layer generic, as pn2_attn_reduce
  if (a.nlayers > 0 && pn2::attn_launch(a, ns, s) != PN2_OK)
    for (int i = 0; i < a.nlayers; ++i) big.l[big.nlayers++] = a.l[i];
  for (int i = 0; i < big.nlayers; ++i) {
    const pn2::AttnLayer& l = big.l[i];
    hipLaunchKernelGGL(pn2::attn_reduce_generic_kernel,
                       dim3(pn2::grid_for((long long)l.G * (l.C / 4))), dim3(pn2::kBlock), 0, s,
                       l.Q, l.K, l.V, l.G, ns, l.C, l.out);
  }
  if (a.nlayers == 0 && big.nlayers == 0) return PN2_OK;
  PN2_RETURN_LAUNCH();
}

int pn2_attn_reduce_grad(const float* Q, const float* K, const float* V, const float* grad_out,
                         int B, int M, int ns, int C, float* grad_Q, float* grad_K,
                         float* grad_V, pn2_stream_t stream) {
  if (B < 0 || M < 0 || ns <= 0 || C < 0 || (C % 4) != 0) return PN2_EINVAL;
  const long long G = (long long)B * M;
  if (G == 0 || C == 0) return PN2_OK;
  if (!Q || !K || !V || !grad_out || !grad_Q || !grad_K || !grad_V || G > INT32_MAX)
    return PN2_EINVAL;
  if ((((uintptr_t)Q | (uintptr_t)K | (uintptr_t)V | (uintptr_t)grad_out | (uintptr_t)grad_Q |
        (uintptr_t)grad_K | (uintptr_t)grad_V) & 15) != 0)
    return PN2_EINVAL;
  hipLaunchKernelGGL(pn2::attn_reduce_grad_kernel, dim3(pn2::grid_for(G * (C / 4))),
                     dim3(pn2::kBlock), 0, (hipStream_t)stream, Q, K, V, grad_out, (int)G, ns, C,
                     grad_Q, grad_K, grad_V);
  PN2_RETURN_LAUNCH();
}

int pn2_group_pool(const float* x, const float* grouped_xyz, int B, int M, int ns, int C,
                   int mode, float* out, pn2_stream_t stream) {
  if (B < 0 || M < 0 || ns <= 0 || C < 0 || mode < PN2_POOL_MAX || mode > PN2_POOL_MAX_AND_AVG)
    return PN2_EINVAL;
  if (mode == PN2_POOL_WEIGHTED_AVG && (ns > 256 || !grouped_xyz)) return PN2_EINVAL;
  const long long G = (long long)B * M;
  if (G == 0 || C == 0) return PN2_OK;
  if (!x || !out || G > INT32_MAX) return PN2_EINVAL;
  hipLaunchKernelGGL(pn2::group_pool_kernel, dim3(pn2::grid_for(G)), dim3(pn2::kBlock), 0,
                     (hipStream_t)stream, x, grouped_xyz, (int)G, ns, C, mode, out);
  PN2_RETURN_LAUNCH();
}

const char* pn2_version(void) { return "pn2hip 0.1 (gfx950)"; }

const char* pn2_strerror(int status) {
  if (status == PN2_OK) return "ok";
  if (status == PN2_EINVAL) return "invalid argument (shape, attribute or null pointer)";
  if (status == PN2_EFAULT)
    return "device fault reported by an earlier sampler launch (see pn2_fault_status)";
  return hipGetErrorString((hipError_t)status);
}

}  // extern "C"
