/*
 * pn2_oracle.c — CPU restatement of the reference's PointNet++ geometric hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This file is the parity checker and the CPU baseline. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the product
 * (libpn2hip.so and the Python package) never calls into it and has no CPU fallback.
 *
 * Every function restates one reference function and cites it (paths relative to
 * /root/reference/pointnet2_tensorflow unless noted). The restatement is pinned two ways
 * (see DESIGN.md §Oracle): against the reference's own CPU code compiled unchanged
 * (oracle/_ref/libref_cpu.so: grouping/test/query_ball_point.cpp, interpolation_3d/
 * interpolate.cpp, tf_interpolate.cpp:57-103) on the golden fixtures of tests/golden/, and
 * against the reference's own CUDA kernels compiled unchanged for gfx950
 * (oracle/_ref/libref_gpu.so: tf_sampling_g.cu, tf_grouping_g.cu) on the GPU box.
 *
 * Arithmetic: plain fp32, compiled with -O2 -ffp-contract=off (no FMA), exactly the
 * non-contracted expression order the reference's C++ writes.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define RFOR _Pragma("omp parallel for schedule(dynamic,1)")

static int g_threads = 1;

void pn2o_set_threads(int n) {
  g_threads = n > 0 ? n : 1;
#ifdef _OPENMP
  omp_set_num_threads(g_threads);
#endif
}
int pn2o_get_threads(void) { return g_threads; }

/* d2 exactly as written in the reference: (x2-x1)*(x2-x1)+(y2-y1)*(y2-y1)+(z2-z1)*(z2-z1),
 * left to right in fp32 (tf_sampling_g.cu:142, query_ball_point.cpp:32, tf_interpolate.cpp:73) */
static inline float sqd(float x2, float y2, float z2, float x1, float y1, float z1) {
  return (x2 - x1) * (x2 - x1) + (y2 - y1) * (y2 - y1) + (z2 - z1) * (z2 - z1);
}

/* CUDA's min(float,float) is fminf (tf_sampling_g.cu:143) */
static inline float cu_min(float a, float b) { return fminf(a, b); }

/* ------------------------------------------------------------------ FPS ---------------- */
/* farthestpointsamplingKernel, tf_sampling_g.cu:105-170, launched <<<32,512>>> (:204):
 * per-thread strided scan with strict '>' (:130-150), then the 512-slot tree reduction
 * (:151-163) whose comparison `dists[i1]<dists[i2]` keeps the left slot on ties.
 * The block/thread structure is emulated literally: 512 virtual threads. */
#define REF_BLOCK 512
void pn2o_fps(const float* xyz, int B, int N, int M, int32_t* idx) {
  RFOR
  for (int b = 0; b < B; ++b) {
    const float* P = xyz + (size_t)b * N * 3;
    int32_t* I = idx + (size_t)b * M;
    if (M <= 0) continue;                   /* :106 */
    float* temp = (float*)malloc(sizeof(float) * (N > 0 ? N : 1));
    float dists[REF_BLOCK];
    int dists_i[REF_BLOCK];
    int old = 0;
    I[0] = old;                             /* :114-116 */
    for (int k = 0; k < N; ++k) temp[k] = 1e38f; /* :117-119 */
    for (int j = 1; j < M; ++j) {           /* :124 */
      float x1 = 0.f, y1 = 0.f, z1 = 0.f;
      if (N > 0) { x1 = P[old * 3 + 0]; y1 = P[old * 3 + 1]; z1 = P[old * 3 + 2]; }
      for (int t = 0; t < REF_BLOCK; ++t) {
        int besti = 0;
        float best = -1;
        for (int k = t; k < N; k += REF_BLOCK) { /* :130 */
          const float td = temp[k];
          const float d = sqd(P[k * 3 + 0], P[k * 3 + 1], P[k * 3 + 2], x1, y1, z1);
          const float d2 = cu_min(d, td);
          if (d2 != td) temp[k] = d2;
          if (d2 > best) { best = d2; besti = k; }
        }
        dists[t] = best;
        dists_i[t] = besti;
      }
      for (int u = 0; (1 << u) < REF_BLOCK; ++u) {   /* :153-163 */
        for (int t = 0; t < (REF_BLOCK >> (u + 1)); ++t) {
          const int i1 = (t * 2) << u, i2 = (t * 2 + 1) << u;
          if (dists[i1] < dists[i2]) { dists[i1] = dists[i2]; dists_i[i1] = dists_i[i2]; }
        }
      }
      old = dists_i[0];                      /* :165 */
      I[j] = old;                            /* :166-167 */
    }
    free(temp);
  }
}

/* gatherpointKernel, tf_sampling_g.cu:172-181 */
void pn2o_gather_point(const float* inp, const int32_t* idx, int B, int N, int M, float* out) {
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < M; ++j) {
      const int a = idx[(size_t)b * M + j];
      for (int c = 0; c < 3; ++c) out[((size_t)b * M + j) * 3 + c] = inp[((size_t)b * N + a) * 3 + c];
    }
}

/* scatteraddpointKernel after cudaMemset, tf_sampling_g.cu:183-192, tf_sampling.cpp:174 */
void pn2o_gather_point_grad(const float* out_g, const int32_t* idx, int B, int N, int M,
                            float* inp_g) {
  memset(inp_g, 0, sizeof(float) * (size_t)B * N * 3);
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < M; ++j) {
      const int a = idx[(size_t)b * M + j];
      for (int c = 0; c < 3; ++c) inp_g[((size_t)b * N + a) * 3 + c] += out_g[((size_t)b * M + j) * 3 + c];
    }
}

/* ------------------------------------------------------------------ grouping ----------- */
/* query_ball_point_cpu, grouping/test/query_ball_point.cpp:19-47, plus pts_cnt from the GPU
 * kernel (tf_grouping_g.cu:34). std::max(a,b) there is (a<b)?b:a. A query with no hit has
 * idx left untouched in the reference; here it is defined as 0 (pn2hip.h). */
void pn2o_ball_query(const float* xyz1, const float* xyz2, int B, int N, int M, float radius,
                     int ns, int32_t* idx, int32_t* pts_cnt) {
  RFOR
  for (int b = 0; b < B; ++b) {
    const float* X1 = xyz1 + (size_t)b * N * 3;
    const float* X2 = xyz2 + (size_t)b * M * 3;
    int32_t* I = idx + (size_t)b * M * ns;
    for (int j = 0; j < M; ++j) {
      int cnt = 0;
      for (int l = 0; l < ns; ++l) I[(size_t)j * ns + l] = 0;
      for (int k = 0; k < N; ++k) {
        if (cnt == ns) break;                                  /* :24-25 */
        const float x2 = X2[j * 3 + 0], y2 = X2[j * 3 + 1], z2 = X2[j * 3 + 2];
        const float x1 = X1[k * 3 + 0], y1 = X1[k * 3 + 1], z1 = X1[k * 3 + 2];
        const float s = sqrtf(sqd(x2, y2, z2, x1, y1, z1));
        const float d = (s < 1e-20f) ? 1e-20f : s;               /* :32 std::max */
        if (d < radius) {                                      /* :33 */
          if (cnt == 0)
            for (int l = 0; l < ns; ++l) I[(size_t)j * ns + l] = k; /* :34-37 */
          I[(size_t)j * ns + cnt] = k;
          cnt += 1;
        }
      }
      pts_cnt[(size_t)b * M + j] = cnt;
    }
  }
}

/* group_point_cpu, query_ball_point.cpp:52-66 */
void pn2o_group_point(const float* points, const int32_t* idx, int B, int N, int C, int M,
                      int ns, float* out) {
  RFOR
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < M; ++j)
      for (int k = 0; k < ns; ++k) {
        const int ii = idx[((size_t)b * M + j) * ns + k];
        for (int l = 0; l < C; ++l)
          out[(((size_t)b * M + j) * ns + k) * C + l] = points[((size_t)b * N + ii) * C + l];
      }
}

/* group_point_grad_cpu, query_ball_point.cpp:70-84 (grad_points zeroed first as
 * tf_grouping.cpp:204 does) */
void pn2o_group_point_grad(const float* grad_out, const int32_t* idx, int B, int N, int C, int M,
                           int ns, float* grad_points) {
  memset(grad_points, 0, sizeof(float) * (size_t)B * N * C);
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < M; ++j)
      for (int k = 0; k < ns; ++k) {
        const int ii = idx[((size_t)b * M + j) * ns + k];
        for (int l = 0; l < C; ++l)
          grad_points[((size_t)b * N + ii) * C + l] += grad_out[(((size_t)b * M + j) * ns + k) * C + l];
      }
}

/* sample_and_group glue, pointnet_util.py:39-56 (SSG) / :186-193 (MSG):
 * grouped_xyz = group_point(xyz, idx) - new_xyz; concat. flags: 1 = use_xyz, 2 = xyz last. */
void pn2o_group_concat(const float* xyz, const float* points, const float* new_xyz,
                       const int32_t* idx, int B, int N, int C, int M, int ns, int flags,
                       float* grouped_xyz, float* new_points) {
  const int use_xyz = flags & 1, xyz_last = (flags >> 1) & 1;
  int Cout;
  if (!points) Cout = 3;
  else if (!use_xyz) Cout = C;
  else Cout = C + 3;
  RFOR
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < M; ++j)
      for (int k = 0; k < ns; ++k) {
        const size_t r = ((size_t)b * M + j) * ns + k;
        const int ii = idx[r];
        float g[3];
        for (int c = 0; c < 3; ++c)
          g[c] = xyz[((size_t)b * N + ii) * 3 + c] - new_xyz[((size_t)b * M + j) * 3 + c];
        if (grouped_xyz) for (int c = 0; c < 3; ++c) grouped_xyz[r * 3 + c] = g[c];
        float* o = new_points + r * Cout;
        if (!points) { for (int c = 0; c < 3; ++c) o[c] = g[c]; continue; }
        const float* p = points + ((size_t)b * N + ii) * C;
        if (!use_xyz) { for (int c = 0; c < C; ++c) o[c] = p[c]; }
        else if (xyz_last) { for (int c = 0; c < C; ++c) o[c] = p[c]; for (int c = 0; c < 3; ++c) o[C + c] = g[c]; }
        else { for (int c = 0; c < 3; ++c) o[c] = g[c]; for (int c = 0; c < C; ++c) o[3 + c] = p[c]; }
      }
}

/* ------------------------------------------------------------------ interpolation ------ */
/* threenn_cpu, tf_interpolate.cpp:60-103 (double bests initialised to 1e40) */
void pn2o_three_nn(const float* xyz1, const float* xyz2, int B, int n, int m, float* dist,
                   int32_t* idx) {
  RFOR
  for (int b = 0; b < B; ++b) {
    const float* X1 = xyz1 + (size_t)b * n * 3;
    const float* X2 = xyz2 + (size_t)b * m * 3;
    for (int j = 0; j < n; ++j) {
      const float x1 = X1[j * 3 + 0], y1 = X1[j * 3 + 1], z1 = X1[j * 3 + 2];
      double best1 = 1e40, best2 = 1e40, best3 = 1e40;
      int besti1 = 0, besti2 = 0, besti3 = 0;
      for (int k = 0; k < m; ++k) {
        const float x2 = X2[k * 3 + 0], y2 = X2[k * 3 + 1], z2 = X2[k * 3 + 2];
        const double d = sqd(x2, y2, z2, x1, y1, z1);
        if (d < best1) { best3 = best2; besti3 = besti2; best2 = best1; besti2 = besti1; best1 = d; besti1 = k; }
        else if (d < best2) { best3 = best2; besti3 = besti2; best2 = d; besti2 = k; }
        else if (d < best3) { best3 = d; besti3 = k; }
      }
      float* D = dist + ((size_t)b * n + j) * 3;
      int32_t* I = idx + ((size_t)b * n + j) * 3;
      D[0] = (float)best1; I[0] = besti1;
      D[1] = (float)best2; I[1] = besti2;
      D[2] = (float)best3; I[2] = besti3;
    }
  }
}

/* threeinterpolate_cpu, tf_interpolate.cpp:107-127 */
void pn2o_three_interpolate(const float* points, const int32_t* idx, const float* weight, int B,
                            int m, int C, int n, float* out) {
  RFOR
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < n; ++j) {
      const size_t r = (size_t)b * n + j;
      const float w1 = weight[r * 3], w2 = weight[r * 3 + 1], w3 = weight[r * 3 + 2];
      const int i1 = idx[r * 3], i2 = idx[r * 3 + 1], i3 = idx[r * 3 + 2];
      const float* P = points + (size_t)b * m * C;
      for (int l = 0; l < C; ++l)
        out[r * C + l] = P[(size_t)i1 * C + l] * w1 + P[(size_t)i2 * C + l] * w2 + P[(size_t)i3 * C + l] * w3;
    }
}

/* threeinterpolate_grad_cpu, tf_interpolate.cpp:131-153 (zeroed first, :246 allocates) */
void pn2o_three_interpolate_grad(const float* grad_out, const int32_t* idx, const float* weight,
                                 int B, int n, int C, int m, float* grad_points) {
  memset(grad_points, 0, sizeof(float) * (size_t)B * m * C);
  for (int b = 0; b < B; ++b)
    for (int j = 0; j < n; ++j) {
      const size_t r = (size_t)b * n + j;
      const float w1 = weight[r * 3], w2 = weight[r * 3 + 1], w3 = weight[r * 3 + 2];
      const int i1 = idx[r * 3], i2 = idx[r * 3 + 1], i3 = idx[r * 3 + 2];
      float* G = grad_points + (size_t)b * m * C;
      for (int l = 0; l < C; ++l) {
        G[(size_t)i1 * C + l] += grad_out[r * C + l] * w1;
        G[(size_t)i2 * C + l] += grad_out[r * C + l] * w2;
        G[(size_t)i3 * C + l] += grad_out[r * C + l] * w3;
      }
    }
}

/* pointnet_util.py:219-222: dist = max(dist,1e-10); norm = sum(1/dist); w = (1/dist)/norm */
void pn2o_idw_weights(const float* dist, int B, int n, float* weight) {
  for (size_t r = 0; r < (size_t)B * n; ++r) {
    float inv[3];
    for (int c = 0; c < 3; ++c) {
      const float d = dist[r * 3 + c];
      inv[c] = 1.0f / (d > 1e-10f ? d : 1e-10f);
    }
    const float norm = (inv[0] + inv[1]) + inv[2];
    for (int c = 0; c < 3; ++c) weight[r * 3 + c] = inv[c] / norm;
  }
}

/* pointnet_fp_module geometry, pointnet_util.py:218-226 */
void pn2o_fp_fused(const float* xyz1, const float* xyz2, const float* points1, int C1,
                   const float* points2, int C2, int B, int n, int m, float* out) {
  float* dist = (float*)malloc(sizeof(float) * (size_t)B * n * 3 + 4);
  float* w = (float*)malloc(sizeof(float) * (size_t)B * n * 3 + 4);
  int32_t* idx = (int32_t*)malloc(sizeof(int32_t) * (size_t)B * n * 3 + 4);
  float* interp = (float*)malloc(sizeof(float) * (size_t)B * n * (C2 > 0 ? C2 : 1));
  pn2o_three_nn(xyz1, xyz2, B, n, m, dist, idx);
  pn2o_idw_weights(dist, B, n, w);
  pn2o_three_interpolate(points2, idx, w, B, m, C2, n, interp);
  const int Cout = C1 + C2;
  for (size_t r = 0; r < (size_t)B * n; ++r) {
    for (int c = 0; c < C2; ++c) out[r * Cout + c] = interp[r * C2 + c];
    for (int c = 0; c < C1; ++c) out[r * Cout + C2 + c] = points1[r * C1 + c];
  }
  free(dist); free(w); free(idx); free(interp);
}

/* ------------------------------------------------------------------ attention ---------- */
/* AttentionLayer.call core, attention_points/attention_scannet/attention_layer.py:35-42,
 * key_dim = output_dim = 4, H = C/4. Head h = flat K/V block [4*ns*h, 4*ns*(h+1)) of the
 * group (tf.reshape reinterpretation, :35-36). */
void pn2o_attn_reduce(const float* Q, const float* K, const float* V, int B, int M, int ns,
                      int C, float* out) {
  const int H = C / 4;
  RFOR
  for (int b = 0; b < B; ++b) {
    float* sc = (float*)malloc(sizeof(float) * (ns > 0 ? ns : 1));
    for (int j = 0; j < M; ++j) {
      const size_t g = (size_t)b * M + j;
      for (int h = 0; h < H; ++h) {
        const float* q = Q + g * C + 4 * h;
        const float* Kh = K + g * ns * C + (size_t)h * 4 * ns;
        const float* Vh = V + g * ns * C + (size_t)h * 4 * ns;
        float mx = -INFINITY;
        for (int s = 0; s < ns; ++s) {
          float v = q[0] * Kh[4 * s];
          v = v + q[1] * Kh[4 * s + 1];
          v = v + q[2] * Kh[4 * s + 2];
          v = v + q[3] * Kh[4 * s + 3];
          sc[s] = v / 2.0f;                         /* :38 / sqrt(4) */
          if (sc[s] > mx) mx = sc[s];
        }
        float sum = 0.f;                            /* :39 softmax */
        for (int s = 0; s < ns; ++s) { sc[s] = expf(sc[s] - mx); sum += sc[s]; }
        for (int d = 0; d < 4; ++d) {               /* :40 */
          float o = 0.f;
          for (int s = 0; s < ns; ++s) o += (sc[s] / sum) * Vh[4 * s + d];
          out[g * C + 4 * h + d] = o;               /* :42 */
        }
      }
    }
    free(sc);
  }
}

/* pooling, pointnet_util.py:130-145; mode 0 max, 1 avg, 2 weighted_avg, 3 max_and_avg */
void pn2o_group_pool(const float* x, const float* gxyz, int B, int M, int ns, int C, int mode,
                     float* out) {
  RFOR
  for (int b = 0; b < B; ++b) {
    float* w = (float*)malloc(sizeof(float) * (ns > 0 ? ns : 1));
    for (int j = 0; j < M; ++j) {
      const size_t g = (size_t)b * M + j;
      const float* X = x + g * ns * C;
      if (mode == 2) {
        float tot = 0.f;
        for (int k = 0; k < ns; ++k) {
          const float* p = gxyz + (g * ns + k) * 3;
          w[k] = expf(-sqrtf(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]) * 5.0f);
          tot += w[k];
        }
        for (int k = 0; k < ns; ++k) w[k] = w[k] / tot;
      }
      for (int c = 0; c < C; ++c) {
        float mx = -INFINITY, sum = 0.f;
        for (int k = 0; k < ns; ++k) {
          const float v = X[(size_t)k * C + c];
          if (v > mx) mx = v;
          sum += (mode == 2) ? v * w[k] : v;
        }
        if (mode == 0) out[g * C + c] = mx;
        else if (mode == 1) out[g * C + c] = sum / (float)ns;
        else if (mode == 2) out[g * C + c] = sum;
        else { out[g * 2 * C + c] = sum / (float)ns; out[g * 2 * C + C + c] = mx; }
      }
    }
    free(w);
  }
}

/* select_top_k / SelectionSort, tf_grouping.py:22-31 -> selection_sort_gpu, tf_grouping_g.cu:83-123,
 * restated literally: each row of dist (B,m,n) is copied with its positions, then for
 * s = 0..k-1 the first position of the minimum over [s, n) (strict '<', :108) is swapped
 * with s (:113-120). outi/out (B,m,n) are the whole permuted rows, as the reference writes. */
void pn2o_selection_sort(const float* dist, int B, int m, int n, int k, int32_t* outi,
                         float* out) {
  RFOR
  for (int b = 0; b < B; ++b) {
    for (int j = 0; j < m; ++j) {
      const size_t r = ((size_t)b * m + j) * n;
      for (int s = 0; s < n; ++s) { out[r + s] = dist[r + s]; outi[r + s] = s; }
      for (int s = 0; s < k && s < n; ++s) {
        int mn = s;
        for (int t = s + 1; t < n; ++t)
          if (out[r + t] < out[r + mn]) mn = t;
        if (mn != s) {
          const float tv = out[r + mn]; out[r + mn] = out[r + s]; out[r + s] = tv;
          const int32_t ti = outi[r + mn]; outi[r + mn] = outi[r + s]; outi[r + s] = ti;
        }
      }
    }
  }
}

/* knn_point, tf_grouping.py:48-73: dist = reduce_sum((xyz1 - xyz2)**2, -1) over the c
 * channels (summed left to right, as Eigen's scalar inner reduction does), then
 * select_top_k(k, dist) and the first k columns: val (B,m,k), idx (B,m,k). */
void pn2o_knn_point(const float* xyz1, const float* xyz2, int B, int n, int m, int c, int k,
                    float* val, int32_t* idx) {
  RFOR
  for (int b = 0; b < B; ++b) {
    float* d = (float*)malloc(sizeof(float) * (n > 0 ? n : 1));
    int32_t* p = (int32_t*)malloc(sizeof(int32_t) * (n > 0 ? n : 1));
    for (int j = 0; j < m; ++j) {
      const float* q = xyz2 + ((size_t)b * m + j) * c;
      for (int t = 0; t < n; ++t) {
        const float* x = xyz1 + ((size_t)b * n + t) * c;
        float acc = 0.f;
        for (int a = 0; a < c; ++a) {
          const float e = x[a] - q[a];
          acc = a == 0 ? e * e : acc + e * e;
        }
        d[t] = acc;
        p[t] = t;
      }
      for (int s = 0; s < k && s < n; ++s) {
        int mn = s;
        for (int t = s + 1; t < n; ++t)
          if (d[t] < d[mn]) mn = t;
        if (mn != s) {
          const float tv = d[mn]; d[mn] = d[s]; d[s] = tv;
          const int32_t ti = p[mn]; p[mn] = p[s]; p[s] = ti;
        }
        val[((size_t)b * m + j) * k + s] = d[s];
        idx[((size_t)b * m + j) * k + s] = p[s];
      }
    }
    free(d);
    free(p);
  }
}

/* ------------------------------------------------------------- prob_sample ------------- */
/* ProbSample (tf_sampling.py:14-23 -> ProbSampleGpuOp tf_sampling.cpp:66-92 ->
 * probsampleLauncher tf_sampling_g.cu:197-201): cumsumKernel (:7-88) then
 * binarysearchKernel (:90-104). The cumsum's fp32 addition order is a fixed function of n,
 * restated here sequentially:
 *  - chunks of 8192 (BlockSize*4, :8, :13); per chunk, 4-element prefixes
 *    v2+=v1, v4+=v3, v3+=v2, v4+=v2 (:18-25), a trailing partial quad summed left to right
 *    and repeated into the padding (:32-40);
 *  - the quad totals scanned by the tree of :43-64 (pairs ((2k+2)<<u)-1 += ((2k+1)<<u)-1 up,
 *    then ((2k+3)<<u)-1 += ((2k+2)<<u)-1 down; the pairs of one level are independent);
 *  - each quad's values += the previous quad's inclusive total (:66-74), out = value +
 *    running sum (:77-79), and the chunk total carried with Kahan compensation (:80-83).
 * binarysearchKernel: q = r * cum[n-1]; r0 = n-1, steps k = base..1 (base = the smallest
 * power of two >= n): if (r0 >= k && cum[r0-k] >= q) r0 -= k. */
#define PS_CHUNK 8192
void pn2o_prob_sample(const float* inp, const float* inpr, int B, int N, int M, int32_t* out) {
  RFOR
  for (int b = 0; b < B; ++b) {
    const float* x = inp + (size_t)b * N;
    float* cum = (float*)malloc(sizeof(float) * (N > 0 ? N : 1));
    float* quad = (float*)malloc(sizeof(float) * PS_CHUNK);
    float* tot = (float*)malloc(sizeof(float) * (PS_CHUNK / 4));
    float run = 0.f, comp = 0.f;
    for (int j = 0; j < N; j += PS_CHUNK) {
      const int len = N - j < PS_CHUNK ? N - j : PS_CHUNK;
      const int len4 = (len + 3) & ~3;
      const int nq = len4 >> 2;
      for (int k = 0; k < len; k += 4) {
        if (k + 3 < len) {
          float v1 = x[j + k], v2 = x[j + k + 1], v3 = x[j + k + 2], v4 = x[j + k + 3];
          v2 += v1;
          v4 += v3;
          v3 += v2;
          v4 += v2;
          quad[k] = v1; quad[k + 1] = v2; quad[k + 2] = v3; quad[k + 3] = v4;
          tot[k >> 2] = v4;
        } else {
          float v = 0.f;
          for (int k2 = k; k2 < len; ++k2) { v += x[j + k2]; quad[k2] = v; }
          for (int k2 = len; k2 < len4; ++k2) quad[k2] = v;
          tot[k >> 2] = v;
        }
      }
      int u = 0;
      for (; (2 << u) <= nq; ++u)
        for (int k = 0; k < (nq >> (u + 1)); ++k)
          tot[(((k << 1) + 2) << u) - 1] += tot[(((k << 1) + 1) << u) - 1];
      for (--u; u >= 0; --u)
        for (int k = 0; k < ((nq - (1 << u)) >> (u + 1)); ++k)
          tot[(((k << 1) + 3) << u) - 1] += tot[(((k << 1) + 2) << u) - 1];
      for (int q = 1; q < nq; ++q)
        for (int e = 0; e < 4; ++e) quad[4 * q + e] += tot[q - 1];
      for (int k = 0; k < len; ++k) cum[j + k] = quad[k] + run;
      const float t = tot[nq - 1] + comp;
      const float r2 = run + t;
      comp = t - (r2 - run);
      run = r2;
    }
    int base = 1;
    while (base < N) base <<= 1;
    for (int i = 0; i < M; ++i) {
      const float q = inpr[(size_t)b * M + i] * cum[N - 1];
      int r = N - 1;
      for (int k = base; k >= 1; k >>= 1)
        if (r >= k && cum[r - k] >= q) r -= k;
      out[(size_t)b * M + i] = r;
    }
    free(cum);
    free(quad);
    free(tot);
  }
}
