// Segmentation head, losses, metric and optimizer kernels.
//
//   head:   Dropout3d (per-(n,c) scale) + 1x1 Conv3d out_conv
//           (reference unet.py:162-163,195-196; dual_encoder.py:83-84,157-158)
//           NDHWC features -> NCDHW fp32 logits (the reference's output layout)
//   loss:   softmax over C + one-hot + per-(b,c) Dice / Tversky sums + CE in one
//           pass; fixed-order finalize; a second pass writes dlogits.
//           DiceLoss losses.py:39-80, DiceCELoss 216-228 (nn.CrossEntropyLoss
//           with optional class weights), TverskyLoss 160-185.
//   metric: argmax over C + per-class integer intersection / union counts
//           (DiceMetric.update, metrics.py:42-67) — integer, exact.
//   optim:  AdamW in torch's single-tensor op order (torch.optim.AdamW, as
//           configured by trainer.py:115-117), over flat parameter buffers.
//   input:  NCDHW fp32 volume -> NDHWC (8-channel padded) engine layout.
#include "mmseg_common.h"

#include <type_traits>

namespace {

constexpr int CMAX = 16;

// -------------------------------------------------------------- input pack
template <typename T>
__global__ void pack_input_kernel(const float* __restrict__ x, int Ctot, int c0, int cnt, long long V, int N,
                                  T* __restrict__ out) {
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    V8<T> o;
    o.zero();
    for (int c = 0; c < cnt; ++c) o.set(c, x[(n * Ctot + c0 + c) * V + v]);
    o.store(out + i * 8);
  }
}

// compact variant for the stem: out[(n*V + v)*cnt + c], no channel padding
template <typename T>
__global__ void pack_input_compact_kernel(const float* __restrict__ x, int Ctot, int c0, int cnt, long long V, int N,
                                          T* __restrict__ out) {
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    for (int c = 0; c < cnt; ++c) out[i * cnt + c] = from_f<T>(x[(n * Ctot + c0 + c) * V + v]);
  }
}

// ----------------------------------------------------------------- head
// logits[n][c][v] = b[c] + sum_ci W[c][ci] * s[n][ci] * x[n,v,ci]
template <typename T>
__global__ void head_fwd_kernel(const T* __restrict__ x, int ldx, int Cin, const float* __restrict__ Wt,
                                const float* __restrict__ bias, const float* __restrict__ dscale, int C, long long V,
                                int N, float* __restrict__ logits) {
  extern __shared__ float sw[];  // C*Cin
  for (int i = threadIdx.x; i < C * Cin; i += blockDim.x) sw[i] = Wt[i];
  __syncthreads();
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    float acc[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = c < C ? bias[c] : 0.f;
    for (int cg = 0; cg < Cin / 8; ++cg) {
      V8<T> a;
      a.load(x + i * ldx + cg * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float xv = a.get(j);
        if (dscale) xv *= dscale[n * Cin + cg * 8 + j];
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) acc[c] = fmaf(sw[c * Cin + cg * 8 + j], xv, acc[c]);
      }
    }
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
      if (c < C) logits[(n * C + c) * V + v] = acc[c];
  }
}

// Same head with the channel-group count CG = Cin / 8 known at compile time and
// U = 4 voxels per thread (i, i + S, i + 2S, i + 3S with S the grid's thread
// count): all U * CG 16-B feature loads are issued before any FMA, and one
// grid of total / (256 U) blocks covers the volume once.  The one-voxel form
// (one block per 256 voxels, each waiting on its weight preload and then on
// 64 B of loads per thread) ran at ~2.2 TB/s.
template <typename T, int CG, int CC>
__global__ __launch_bounds__(256) void head_fwd_u_kernel(const T* __restrict__ x, int ldx,
                                                         const float* __restrict__ Wt, const float* __restrict__ bias,
                                                         const float* __restrict__ dscale, long long V, int N,
                                                         float* __restrict__ logits) {
  constexpr int Cin = CG * 8, U = 4;
  __shared__ float sw[CC * Cin];
  for (int i = threadIdx.x; i < CC * Cin; i += blockDim.x) sw[i] = Wt[i];
  const long long total = (long long)N * V;
  const long long S = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  V8<T> a[U][CG];
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (i0 + u * S < total)
#pragma unroll
      for (int cg = 0; cg < CG; ++cg) a[u][cg].load(x + (i0 + u * S) * ldx + cg * 8);
  __syncthreads();
  float acc[U][CC];
#pragma unroll
  for (int c = 0; c < CC; ++c) {
    const float b = bias[c];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u][c] = b;
  }
  // weights outer (read once from LDS per (ci, c)), the U voxels inner
#pragma unroll
  for (int cg = 0; cg < CG; ++cg)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        xv[u] = a[u][cg].get(j);
        if (dscale && i0 + u * S < total) xv[u] *= dscale[((i0 + u * S) / V) * Cin + cg * 8 + j];
      }
#pragma unroll
      for (int c = 0; c < CC; ++c) {
        const float w = sw[c * Cin + cg * 8 + j];
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u][c] = fmaf(w, xv[u], acc[u][c]);
      }
    }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = i0 + u * S;
    if (i >= total) break;
    const long long n = i / V, v = i - n * V;
#pragma unroll
    for (int c = 0; c < CC; ++c) logits[(n * CC + c) * V + v] = acc[u][c];
  }
}

// dx[n,v,ci] = s[n][ci] * sum_c dlog[n][c][v] * W[c][ci]
template <typename T>
__global__ void head_dgrad_kernel(const float* __restrict__ dlog, const float* __restrict__ Wt,
                                  const float* __restrict__ dscale, int C, int Cin, long long V, int N,
                                  T* __restrict__ dx, int lddx) {
  extern __shared__ float sw[];
  for (int i = threadIdx.x; i < C * Cin; i += blockDim.x) sw[i] = Wt[i];
  __syncthreads();
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    float d[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) d[c] = c < C ? dlog[(n * C + c) * V + v] : 0.f;
    for (int cg = 0; cg < Cin / 8; ++cg) {
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = cg * 8 + j;
        float a = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) a = fmaf(d[c], sw[c * Cin + ci], a);
        if (dscale) a *= dscale[n * Cin + ci];
        o.set(j, a);
      }
      o.store(dx + i * lddx + cg * 8);
    }
  }
}


// Quad-per-voxel head data gradient: lane q of a 4-lane quad writes the 8-channel groups q, q+4, ... of its
// voxel, so a wave stores 16 voxels x 64 contiguous bytes with 16-B lanes (71 us vs 86 us for the
// one-voxel-per-lane form at 96^3 B=2; the same quad form of the forward measured slower and is not used).
template <typename T>
__global__ __launch_bounds__(256) void head_dgrad_q_kernel(const float* __restrict__ dlog,
                                                           const float* __restrict__ Wt,
                                                           const float* __restrict__ dscale, int C, int Cin,
                                                           long long V, int N, T* __restrict__ dx, int lddx) {
  extern __shared__ float sw[];
  for (int i = threadIdx.x; i < C * Cin; i += blockDim.x) sw[i] = Wt[i];
  __syncthreads();
  const int q = threadIdx.x & 3, C8 = Cin >> 3;
  const long long total = (long long)N * V;
  for (long long i = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 2; i < total;
       i += ((long long)gridDim.x * blockDim.x) >> 2) {
    const long long n = i / V, v = i - n * V;
    float d[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) d[c] = c < C ? dlog[(n * C + c) * V + v] : 0.f;
    for (int cg = q; cg < C8; cg += 4) {
      V8<T> o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int ci = cg * 8 + j;
        float a = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) a = fmaf(d[c], sw[c * Cin + ci], a);
        if (dscale) a *= dscale[n * Cin + ci];
        o.set(j, a);
      }
      o.store(dx + i * lddx + cg * 8);
    }
  }
}

// partial dW[c][ci] and db[c] per voxel chunk (block), fixed order.
// thread = (voxel lane, 8-channel group): vectorised x loads, 8x8 register tile per class chunk.
template <typename T>
__global__ __launch_bounds__(256) void head_wgrad_partial(const T* __restrict__ x, int ldx, const float* __restrict__ dlog,
                                   const float* __restrict__ dscale, int C, int Cin, long long V, int N,
                                   long long vpc, float* __restrict__ part) {
  __shared__ float red[256 * 8 + 4];
  const int C8 = Cin >> 3;
  const int lanes_v = 256 / C8;
  const int tid = threadIdx.x;
  const int cg = tid % C8, vl = tid / C8;
  const long long total = (long long)N * V;
  const long long e0 = (long long)blockIdx.x * vpc;
  long long e1 = e0 + vpc;
  if (e1 > total) e1 = total;
  const int npairs = C * Cin + C;
  for (int c0 = 0; c0 < C; c0 += 8) {
    float acc[8][8], bacc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bacc[k] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[k][j] = 0.f;
    }
    if (vl < lanes_v) {
      // U voxels per step: their feature and dlogits loads are issued before any FMA
      constexpr int U = 2;
      for (long long eb = e0 + vl; eb < e1; eb += U * lanes_v) {
        V8<T> a[U];
        float dd[U][8];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long e = eb + u * lanes_v;
          if (e < e1) {
            const long long n = e / V, v = e - n * V;
            a[u].load(x + e * ldx + cg * 8);
#pragma unroll
            for (int k = 0; k < 8; ++k) dd[u][k] = c0 + k < C ? dlog[(n * C + c0 + k) * V + v] : 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const long long e = eb + u * lanes_v;
          if (e >= e1) break;
          const long long n = e / V;
          float xv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) xv[j] = dscale ? a[u].get(j) * dscale[n * Cin + cg * 8 + j] : a[u].get(j);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float d = dd[u][k];
            bacc[k] += d;
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[k][j] = fmaf(d, xv[j], acc[k][j]);
          }
        }
      }
    }
    if ((C8 & (C8 - 1)) == 0 && C8 <= 32) {
      // power-of-two channel groups: shuffle tree over the voxel lanes of each wave (fixed order), then
      // the 4 waves in order through LDS (the serial 64-lane LDS sweep per class cost ~2 us per block)
      for (int o = 32; o >= C8; o >>= 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          bacc[k] += __shfl_down(bacc[k], o, 64);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[k][j] += __shfl_down(acc[k][j], o, 64);
        }
      }
      const int lane = tid & 63, wave = tid >> 6;
      for (int k = 0; k < 8 && c0 + k < C; ++k) {
        __syncthreads();
        if (lane < C8) {
#pragma unroll
          for (int j = 0; j < 8; ++j) red[(wave * C8 + lane) * 8 + j] = acc[k][j];
          if (lane == 0) red[4 * 32 * 8 + wave] = bacc[k];
        }
        __syncthreads();
        for (int ci = tid; ci < Cin; ci += 256) {
          const int g = ci >> 3, j = ci & 7;
          float sacc = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) sacc += red[(w * C8 + g) * 8 + j];
          part[(long long)blockIdx.x * npairs + (c0 + k) * Cin + ci] = sacc;
        }
        if (tid == 0) {
          float sacc = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) sacc += red[4 * 32 * 8 + w];
          part[(long long)blockIdx.x * npairs + C * Cin + c0 + k] = sacc;
        }
      }
      continue;
    }
    for (int k = 0; k < 8 && c0 + k < C; ++k) {
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 8; ++j) red[tid * 8 + j] = acc[k][j];
      __syncthreads();
      for (int ci = tid; ci < Cin; ci += 256) {
        const int g = ci >> 3, j = ci & 7;
        float sacc = 0.f;
        for (int l = 0; l < lanes_v; ++l) sacc += red[(l * C8 + g) * 8 + j];
        part[(long long)blockIdx.x * npairs + (c0 + k) * Cin + ci] = sacc;
      }
      __syncthreads();
      red[tid] = (cg == 0 && vl < lanes_v) ? bacc[k] : 0.f;
      __syncthreads();
      if (tid == 0) {
        float sacc = 0.f;
        for (int l = 0; l < lanes_v; ++l) sacc += red[l * C8];
        part[(long long)blockIdx.x * npairs + C * Cin + c0 + k] = sacc;
      }
    }
  }
}

// one wave per output (C*Cin weights + C biases): lanes stride over the block
// partials, fixed shuffle tree -> deterministic, 64 loads in flight per output
__global__ void head_wgrad_reduce(const float* __restrict__ part, int nblk, int C, int Cin, float* __restrict__ gW,
                                  float* __restrict__ gb, int accumulate) {
  const int npairs = C * Cin + C;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= npairs) return;
  float a = 0.f;
  for (int b = lane; b < nblk; b += 64) a += part[(long long)b * npairs + p];
  a = wave_sum(a);
  if (lane == 0) {
    float* dst = p < C * Cin ? gW + p : gb + (p - C * Cin);
    *dst = accumulate ? *dst + a : a;
  }
}

// ----------------------------------------------------------------- losses
struct LossCfg {
  int type;             // 0 = dice/ce family, 1 = tversky, 2 = focal (alpha = gamma; region weight 0)
  float dice_w, ce_w;   // weights of the region term and the CE term
  float smooth, alpha, beta;
  int include_bg;
  const float* cw;      // CE class weights [C] or null
};

// Label validity (the reference raises in F.one_hot / cross_entropy on a label outside [0, C)): such a
// voxel contributes nothing and is counted; the finalize pass then makes the loss NaN and publishes the
// count at coef[2NC+1] for the host to raise on.  Pure CE (region weight 0) skips torch's default
// ignore_index -100 without counting it, as nn.CrossEntropyLoss does.
__device__ __forceinline__ int label_state(int y, int C, const LossCfg& cfg) {
  if ((unsigned)y < (unsigned)C) return 0;                 // valid
  return (y == -100 && cfg.type == 0 && cfg.dice_w == 0.f) ? 1 : 2;   // 1 = ignored, 2 = invalid
}

// per (n, chunk): [P_c][I_c][T_c] (3C) + ce_num + ce_den + invalid-label count
template <typename LT, int CC>
__global__ __launch_bounds__(256) void loss_stats_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int Crt,
                                  long long V, long long vpc, LossCfg cfg, float* __restrict__ part) {
  // CC > 0: class count known at compile time (U voxels in flight); CC = 0: runtime C, one voxel at a time
  const int C = CC > 0 ? CC : Crt;
  constexpr int NC = CC > 0 ? CC : CMAX;
  const int n = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  float P[NC], I[NC], Tc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) P[c] = I[c] = Tc[c] = 0.f;
  float ce = 0.f, cden = 0.f, bad = 0.f;
  const long long v0 = (long long)chunk * vpc;
  long long v1 = v0 + vpc;
  if (v1 > V) v1 = V;
  const float* L = logits + (long long)n * C * V;
  // U voxels per thread per step: their C logits and labels are loaded before any is consumed
  constexpr int U = CC > 0 ? 4 : 1;
  for (long long vb = v0 + threadIdx.x; vb < v1; vb += U * blockDim.x) {
  float zu[U][NC];
  int yu[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long v = vb + u * blockDim.x;
    if (v < v1) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) zu[u][c] = L[c * V + v];
      yu[u] = (int)labels[(long long)n * V + v];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (vb + u * blockDim.x >= v1) break;
    const int y = yu[u];
    const int ls = label_state(y, C, cfg);
    if (ls) {
      bad += ls == 2 ? 1.f : 0.f;
      continue;
    }
    float z[NC];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        z[c] = zu[u][c];
        mx = fmaxf(mx, z[c]);
      }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) se += expf(z[c] - mx);
    const float lse = mx + logf(se);
    const float inv = 1.f / se;
    float zy = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        const float p = expf(z[c] - mx) * inv;
        P[c] += p;
        if (c == y) {
          I[c] += p;
          Tc[c] += 1.f;
          zy = z[c];
        }
      }
    const float wy = cfg.cw ? cfg.cw[y] : 1.f;
    if (cfg.type == 2) {   // focal (losses.py:116-121): (1 - exp(-ce_i))^gamma * ce_i, plain mean over voxels
      const float cei = wy * (lse - zy);
      const float pt = expf(-cei);
      ce += powf(1.f - pt, cfg.alpha) * cei;
      cden += 1.f;
    } else {
      ce = fmaf(wy, lse - zy, ce);
      cden += wy;
    }
  }
  }
  __shared__ float red[4][3 * CMAX + 3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int c = 0; c < C; ++c) {
    float a = wave_sum(P[c]), b = wave_sum(I[c]), d = wave_sum(Tc[c]);
    if (lane == 0) {
      red[wave][c] = a;
      red[wave][C + c] = b;
      red[wave][2 * C + c] = d;
    }
  }
  {
    float a = wave_sum(ce), b = wave_sum(cden), d = wave_sum(bad);
    if (lane == 0) {
      red[wave][3 * C] = a;
      red[wave][3 * C + 1] = b;
      red[wave][3 * C + 2] = d;
    }
  }
  __syncthreads();
  const int nv = 3 * C + 3;
  for (int k = threadIdx.x; k < nv; k += blockDim.x)
    part[((long long)n * nchunk + chunk) * nv + k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// one block: loss scalar + per-(n,c) dp coefficients (dp = a*t + b) + ce scale
// 1024 threads.  Phase 1: wave w sums quantity (n, q) over the chunks (lanes
// stride the chunks, fixed fp64 shuffle tree).  Phase 2: thread e = (n, c)
// forms the region term and its gradient coefficients.  Phase 3: thread 0
// adds the N*C region terms and the CE sums in index order.
__global__ void loss_finalize_kernel(const float* __restrict__ part, int N, int C, int nchunk, LossCfg cfg,
                                     float* __restrict__ loss_out, float* __restrict__ coef) {
  extern __shared__ double S[];           // [N*nv] sums, then [N*C] region terms
  const int nv = 3 * C + 3;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nwave = blockDim.x >> 6;
  for (int pr = wave; pr < N * nv; pr += nwave) {
    const int n = pr / nv, q = pr - n * nv;
    double a = 0.0;
    for (int k = lane; k < nchunk; k += 64) a += part[((long long)n * nchunk + k) * nv + q];
    a = wave_sum_d(a);
    if (lane == 0) S[pr] = a;
  }
  __syncthreads();
  double* R = S + N * nv;
  const int c0 = (cfg.type == 0 && !cfg.include_bg) ? 1 : 0;
  const double nterms = (double)N * (C - c0);
  for (int e = threadIdx.x; e < N * C; e += blockDim.x) {
    const int n = e / C, c = e - n * C;
    const double P = S[n * nv + c], I = S[n * nv + C + c], T = S[n * nv + 2 * C + c];
    double a = 0.0, b = 0.0, region = 0.0;
    const double s = cfg.smooth;
    if (c >= c0) {
      if (cfg.type == 0) {
        const double U = P + T;
        const double dice = (2.0 * I + s) / (U + s);
        region = 1.0 - dice;
        a = -(2.0 / (U + s)) / nterms;
        b = ((2.0 * I + s) / ((U + s) * (U + s))) / nterms;
      } else {
        const double fp = P - I, fn = T - I;
        const double num = I + s;
        const double den = I + cfg.alpha * fp + cfg.beta * fn + s;
        region = 1.0 - num / den;
        a = -((den - num * (1.0 - cfg.alpha - cfg.beta)) / (den * den)) / nterms;
        b = (num * cfg.alpha / (den * den)) / nterms;
      }
    }
    R[e] = region;
    coef[e * 2 + 0] = (float)(a * cfg.dice_w);
    coef[e * 2 + 1] = (float)(b * cfg.dice_w);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = 0.0, ce = 0.0, den = 0.0, bad = 0.0;
    for (int e = 0; e < N * C; ++e) r += R[e];
    for (int n = 0; n < N; ++n) {
      ce += S[n * nv + 3 * C];
      den += S[n * nv + 3 * C + 1];
      bad += S[n * nv + 3 * C + 2];
    }
    const double lv = cfg.dice_w * (r / nterms) + cfg.ce_w * (ce / den);
    loss_out[0] = bad > 0.0 ? __builtin_nanf("") : (float)lv;
    coef[2 * N * C] = (float)(cfg.ce_w / den);   // CE gradient scale
    coef[2 * N * C + 1] = (float)bad;            // labels outside [0, C): the host raises on a non-zero count
  }
}

// dlogits = gout * [ p*(dp - sum p dp) + ce_scale * w_y * (p - t) ]
template <typename LT, int CC>
__global__ __launch_bounds__(256) void loss_bwd_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int Crt, long long V,
                                int N, LossCfg cfg, const float* __restrict__ coef, const float* __restrict__ gout,
                                float gconst, float* __restrict__ dlogits) {
  // CC > 0: class count known at compile time (U voxels in flight); CC = 0: runtime C, one voxel at a time
  const int C = CC > 0 ? CC : Crt;
  constexpr int NC = CC > 0 ? CC : CMAX;
  const long long total = (long long)N * V;
  const float g = gout ? gout[0] * gconst : gconst;
  const float ces = coef[2 * N * C];
  // U voxels per thread (i, i + S, ...): logits and labels of all U loaded before any is consumed
  constexpr int U = CC > 0 ? 4 : 1;
  const long long S = (long long)gridDim.x * blockDim.x;
  for (long long ib = (long long)blockIdx.x * blockDim.x + threadIdx.x; ib < total; ib += U * S) {
  float zu[U][NC];
  int yu[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = ib + u * S;
    if (i < total) {
      const long long n = i / V, v = i - n * V;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) zu[u][c] = logits[(n * C + c) * V + v];
      yu[u] = (int)labels[i];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = ib + u * S;
    if (i >= total) break;
    const long long n = i / V, v = i - n * V;
    const int y = yu[u];
    if (label_state(y, C, cfg)) {     // ignored / invalid label: no gradient through this voxel
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C) dlogits[(n * C + c) * V + v] = 0.f;
      continue;
    }
    float z[NC], p[NC];
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        z[c] = zu[u][c];
        mx = fmaxf(mx, z[c]);
      }
    float se = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        p[c] = expf(z[c] - mx);
        se += p[c];
      }
    const float inv = 1.f / se;
    float wy = cfg.cw ? cfg.cw[y] : 1.f;
    if (cfg.type == 2) {   // focal: d f_i / d ce_i = gamma (1-pt)^(gamma-1) pt ce_i + (1-pt)^gamma, ce_i = w_y (lse - z_y)
      float zy = 0.f;
#pragma unroll
      for (int c = 0; c < NC; ++c)
        if (c < C && c == y) zy = z[c];
      const float cei = wy * (mx + logf(se) - zy);
      const float pt = expf(-cei), q = 1.f - pt, gm = cfg.alpha;
      const float dfd = (q > 0.f ? gm * powf(q, gm - 1.f) * pt * cei : 0.f) + powf(q, gm);
      wy *= dfd;
    }
    float dp[NC];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        p[c] *= inv;
        const float t = c == y ? 1.f : 0.f;
        const float* cf = coef + ((long long)n * C + c) * 2;
        dp[c] = cf[0] * t + cf[1];
        s = fmaf(p[c], dp[c], s);
      }
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (c < C) {
        const float t = c == y ? 1.f : 0.f;
        const float d = p[c] * (dp[c] - s) + ces * wy * (p[c] - t);
        dlogits[(n * C + c) * V + v] = g * d;
      }
  }
  }
}

// -------------------------------------------------------------- metric
// counts[0..C) intersection, [C..2C) pred count, [2C..3C) target count
template <typename LT>
__global__ void dice_counts_kernel(const float* __restrict__ logits, const LT* __restrict__ labels, int C, long long V,
                                   int N, unsigned long long* __restrict__ counts, LT* __restrict__ pred_out) {
  __shared__ unsigned int sc[3 * CMAX];
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x) sc[k] = 0;
  __syncthreads();
  const long long total = (long long)N * V;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long n = i / V, v = i - n * V;
    const float* L = logits + n * C * V;
    int best = 0;
    float bv = L[v];
    for (int c = 1; c < C; ++c) {
      const float z = L[c * V + v];
      if (z > bv || (z != z && bv == bv)) {  // first maximum; NaN counts as maximal (torch.argmax)
        bv = z;
        best = c;
      }
    }
    const int y = (int)labels[i];
    if (pred_out) pred_out[i] = (LT)best;
    atomicAdd(&sc[C + best], 1u);
    if (y >= 0 && y < C) {
      atomicAdd(&sc[2 * C + y], 1u);
      if (y == best) atomicAdd(&sc[y], 1u);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x)
    if (sc[k]) atomicAdd(&counts[k], (unsigned long long)sc[k]);
}

template <typename PT, typename LT>
__global__ void dice_counts_idx_kernel(const PT* __restrict__ pred, const LT* __restrict__ labels, int C,
                                       long long total, unsigned long long* __restrict__ counts) {
  __shared__ unsigned int sc[3 * CMAX];
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x) sc[k] = 0;
  __syncthreads();
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int p = (int)pred[i], y = (int)labels[i];
    if (p >= 0 && p < C) atomicAdd(&sc[C + p], 1u);
    if (y >= 0 && y < C) {
      atomicAdd(&sc[2 * C + y], 1u);
      if (y == p) atomicAdd(&sc[y], 1u);
    }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 3 * C; k += blockDim.x)
    if (sc[k]) atomicAdd(&counts[k], (unsigned long long)sc[k]);
}

// ------------------------------------------------------------------ AdamW
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long long n, float decay, float beta1, float omb1, float beta2,
                             float omb2, float eps, float step_size, float bc2_sqrt) {
#pragma clang fp contract(off)
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float pv = p[i];
    const float gv = g[i];
    pv = pv * decay;                          // param.mul_(1 - lr * wd)
    float mv = m[i];
    mv = omb1 < 0.5f ? mv + omb1 * (gv - mv)  // exp_avg.lerp_(grad, 1 - beta1)
                     : gv - (gv - mv) * (1.f - omb1);
    float vv = v[i];
    vv = vv * beta2 + (omb2 * gv) * gv;       // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    pv = pv + (-step_size) * (mv / denom);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

int grid_for(long long total) {
  long long b = (total + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (int)b;
}

int loss_chunks(long long V, long long* vpc) {
  long long nch = (V + 2047) / 2048;
  if (nch > 1024) nch = 1024;
  if (nch < 1) nch = 1;
  *vpc = (V + nch - 1) / nch;
  return (int)((V + *vpc - 1) / *vpc);
}

}  // namespace

extern "C" {

int mmseg_pack_input(const float* x, int Ctot, int c0, int cnt, int N, long long V, void* out, int dtype,
                     void* stream) {
  MMSEG_REQUIRE(cnt >= 1 && cnt <= 8, "pack_input: 1..8 channels per pack (got %d)", cnt);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V);
  if (dtype == MMSEG_BF16)
    hipLaunchKernelGGL(pack_input_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N, (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_input_kernel<float>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N, (float*)out);
  return mmseg::check_launch("pack_input");
}

int mmseg_pack_input_compact(const float* x, int Ctot, int c0, int cnt, int N, long long V, void* out, int dtype,
                             void* stream) {
  MMSEG_REQUIRE(cnt >= 1 && cnt <= 4, "pack_input_compact: 1..4 channels (got %d)", cnt);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V);
  if (dtype == MMSEG_BF16)
    hipLaunchKernelGGL(pack_input_compact_kernel<bf16_t>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N,
                       (bf16_t*)out);
  else
    hipLaunchKernelGGL(pack_input_compact_kernel<float>, dim3(grid), dim3(256), 0, s, x, Ctot, c0, cnt, V, N,
                       (float*)out);
  return mmseg::check_launch("pack_input_compact");
}

int mmseg_head_fwd(const void* x, int ldx, int Cin, const float* W, const float* b, const float* dscale, int C, int N,
                   long long V, float* logits, int dtype, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX && Cin % 8 == 0, "head: 1 <= C <= %d, Cin%%8 == 0", CMAX);
  hipStream_t s = (hipStream_t)stream;
  const int ugrid = (int)ceil_div((long long)N * V, 256LL * 4);
  auto run_u = [&](auto tag, auto cg_c, auto cc_c) -> bool {
    using T = decltype(tag);
    constexpr int CG = decltype(cg_c)::value, CC = decltype(cc_c)::value;
    if (Cin != CG * 8 || C != CC) return false;
    hipLaunchKernelGGL((head_fwd_u_kernel<T, CG, CC>), dim3(ugrid), dim3(256), 0, s, (const T*)x, ldx, W, b, dscale,
                       V, N, logits);
    return true;
  };
  // the configs' heads: 32 (UNet / DualEncoder) or 48 (SwinUNETR fs=48) input channels, 3 / 6 / 7 classes
  auto try_cc = [&](auto tag, auto cg_c) {
    return run_u(tag, cg_c, std::integral_constant<int, 3>{}) || run_u(tag, cg_c, std::integral_constant<int, 6>{}) ||
           run_u(tag, cg_c, std::integral_constant<int, 7>{});
  };
  auto try_u = [&](auto tag) {
    return try_cc(tag, std::integral_constant<int, 4>{}) || try_cc(tag, std::integral_constant<int, 6>{});
  };
  if (ldx % 8 == 0 && (dtype == MMSEG_BF16 ? try_u(bf16_t{}) : try_u(float{})))
    return mmseg::check_launch("head_fwd");
  const int grid = grid_for((long long)N * V);
  const size_t shm = (size_t)C * Cin * sizeof(float);
  if (dtype == MMSEG_BF16)
    hipLaunchKernelGGL(head_fwd_kernel<bf16_t>, dim3(grid), dim3(256), shm, s, (const bf16_t*)x, ldx, Cin, W, b, dscale,
                       C, V, N, logits);
  else
    hipLaunchKernelGGL(head_fwd_kernel<float>, dim3(grid), dim3(256), shm, s, (const float*)x, ldx, Cin, W, b, dscale,
                       C, V, N, logits);
  return mmseg::check_launch("head_fwd");
}

long long mmseg_head_ws_floats(int C, int Cin, int N, long long V) {
  const long long nblk = 2048;
  return nblk * (C * Cin + C);
}

int mmseg_head_bwd(const void* x, int ldx, int Cin, const float* W, const float* dscale, int C, int N, long long V,
                   const float* dlogits, void* dx, int lddx, float* gW, float* gb, float* ws, int accumulate, int dtype,
                   void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX && Cin % 8 == 0 && Cin <= 2048, "head_bwd: shape");
  hipStream_t s = (hipStream_t)stream;
  const long long total = (long long)N * V;
  const int qgrid = grid_for(4 * total);
  const size_t shm = (size_t)C * Cin * sizeof(float);
  long long nblk = 2048;
  long long vpc = ((total + nblk - 1) / nblk + 63) / 64 * 64;
  nblk = (total + vpc - 1) / vpc;
  const size_t shm2 = 0;
  // weight-gradient partials first: dx may alias x (the engine reuses the feature buffer)
  if (dtype == MMSEG_BF16) {
    hipLaunchKernelGGL(head_wgrad_partial<bf16_t>, dim3((int)nblk), dim3(256), shm2, s, (const bf16_t*)x, ldx, dlogits,
                       dscale, C, Cin, V, N, vpc, ws);
    if (dx)
      hipLaunchKernelGGL(head_dgrad_q_kernel<bf16_t>, dim3(qgrid), dim3(256), shm, s, dlogits, W, dscale, C, Cin, V,
                         N, (bf16_t*)dx, lddx);
  } else {
    hipLaunchKernelGGL(head_wgrad_partial<float>, dim3((int)nblk), dim3(256), shm2, s, (const float*)x, ldx, dlogits,
                       dscale, C, Cin, V, N, vpc, ws);
    if (dx)
      hipLaunchKernelGGL(head_dgrad_q_kernel<float>, dim3(qgrid), dim3(256), shm, s, dlogits, W, dscale, C, Cin, V, N,
                         (float*)dx, lddx);
  }
  if (mmseg::check_launch("head_bwd")) return 1;
  hipLaunchKernelGGL(head_wgrad_reduce, dim3(ceil_div(C * Cin + C, 4)), dim3(256), 0, s, ws, (int)nblk, C, Cin, gW,
                     gb, accumulate);
  return mmseg::check_launch("head_wgrad_reduce");
}

long long mmseg_loss_ws_floats(int N, int C, long long V) {
  long long vpc;
  int nch = loss_chunks(V, &vpc);
  return (long long)N * nch * (3 * C + 3) + 2LL * N * C + 2;
}

// label_bytes: 8 (int64, the reference's dtype) or 1 (uint8)
int mmseg_loss_fwd(const float* logits, const void* labels, int label_bytes, int N, int C, long long V, int type,
                   float dice_w, float ce_w, float smooth, float alpha, float beta, int include_bg,
                   const float* class_w, float* loss_out, float* ws, void* stream) {
  MMSEG_REQUIRE(C >= 2 && C <= CMAX, "loss: 2 <= C <= %d", CMAX);
  MMSEG_REQUIRE(label_bytes == 8 || label_bytes == 1, "loss: labels must be int64 or uint8");
  LossCfg cfg{type, dice_w, ce_w, smooth, alpha, beta, include_bg, class_w};
  long long vpc;
  const int nch = loss_chunks(V, &vpc);
  float* part = ws;
  float* coef = ws + (long long)N * nch * (3 * C + 3);
  hipStream_t s = (hipStream_t)stream;
  auto stats = [&](auto lt, auto cc) {
    using LT = decltype(lt);
    hipLaunchKernelGGL((loss_stats_kernel<LT, decltype(cc)::value>), dim3(nch, N), dim3(256), 0, s, logits,
                       (const LT*)labels, C, V, vpc, cfg, part);
  };
  auto stats_c = [&](auto lt) {
    if (C == 3) stats(lt, std::integral_constant<int, 3>{});
    else if (C == 6) stats(lt, std::integral_constant<int, 6>{});
    else if (C == 7) stats(lt, std::integral_constant<int, 7>{});
    else stats(lt, std::integral_constant<int, 0>{});
  };
  if (label_bytes == 8) stats_c(int64_t{});
  else stats_c(uint8_t{});
  if (mmseg::check_launch("loss_stats")) return 1;
  const size_t shm = sizeof(double) * ((size_t)N * (3 * C + 3) + (size_t)N * C);
  MMSEG_REQUIRE(shm <= 64 * 1024, "loss: batch too large for the finalize pass (N=%d, C=%d)", N, C);
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(1024), shm, s, part, N, C, nch, cfg, loss_out, coef);
  return mmseg::check_launch("loss_finalize");
}

// Must follow mmseg_loss_fwd with the same ws.  gout (device scalar) may be null.
int mmseg_loss_bwd(const float* logits, const void* labels, int label_bytes, int N, int C, long long V, int type,
                   float dice_w, float ce_w, float smooth, float alpha, float beta, int include_bg,
                   const float* class_w, const float* gout, float gconst, float* dlogits, const float* ws,
                   void* stream) {
  LossCfg cfg{type, dice_w, ce_w, smooth, alpha, beta, include_bg, class_w};
  long long vpc;
  const int nch = loss_chunks(V, &vpc);
  const float* coef = ws + (long long)N * nch * (3 * C + 3);
  hipStream_t s = (hipStream_t)stream;
  auto bwd = [&](auto lt, auto cc) {
    using LT = decltype(lt);
    constexpr int CC = decltype(cc)::value;
    const int grid = grid_for(CC > 0 ? ceil_div((long long)N * V, 4) : (long long)N * V);
    hipLaunchKernelGGL((loss_bwd_kernel<LT, CC>), dim3(grid), dim3(256), 0, s, logits, (const LT*)labels, C, V, N, cfg,
                       coef, gout, gconst, dlogits);
  };
  auto bwd_c = [&](auto lt) {
    if (C == 3) bwd(lt, std::integral_constant<int, 3>{});
    else if (C == 6) bwd(lt, std::integral_constant<int, 6>{});
    else if (C == 7) bwd(lt, std::integral_constant<int, 7>{});
    else bwd(lt, std::integral_constant<int, 0>{});
  };
  if (label_bytes == 8) bwd_c(int64_t{});
  else bwd_c(uint8_t{});
  return mmseg::check_launch("loss_bwd");
}

// counts: 3*C uint64 (must be zeroed by the caller, accumulates); pred_out optional (same dtype as labels)
int mmseg_dice_counts(const float* logits, const void* labels, int label_bytes, int N, int C, long long V,
                      unsigned long long* counts, void* pred_out, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX, "dice_counts: C <= %d", CMAX);
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for((long long)N * V) > 2048 ? 2048 : grid_for((long long)N * V);
  if (label_bytes == 8)
    hipLaunchKernelGGL(dice_counts_kernel<int64_t>, dim3(grid), dim3(256), 0, s, logits, (const int64_t*)labels, C, V,
                       N, counts, (int64_t*)pred_out);
  else
    hipLaunchKernelGGL(dice_counts_kernel<uint8_t>, dim3(grid), dim3(256), 0, s, logits, (const uint8_t*)labels, C, V,
                       N, counts, (uint8_t*)pred_out);
  return mmseg::check_launch("dice_counts");
}

// counts from class-index masks (DiceMetric.update(pred, target), metrics.py:42-67); int64 or uint8 masks
int mmseg_dice_counts_idx(const void* pred, int pred_bytes, const void* labels, int label_bytes, long long total, int C,
                          unsigned long long* counts, void* stream) {
  MMSEG_REQUIRE(C >= 1 && C <= CMAX && (pred_bytes == 8 || pred_bytes == 1) && (label_bytes == 8 || label_bytes == 1),
                "dice_counts_idx: bad args");
  hipStream_t s = (hipStream_t)stream;
  const int grid = grid_for(total) > 2048 ? 2048 : grid_for(total);
#define DCI(PT, LT) \
  hipLaunchKernelGGL((dice_counts_idx_kernel<PT, LT>), dim3(grid), dim3(256), 0, s, (const PT*)pred, (const LT*)labels, C, total, counts)
  if (pred_bytes == 8 && label_bytes == 8) DCI(int64_t, int64_t);
  else if (pred_bytes == 8) DCI(int64_t, uint8_t);
  else if (label_bytes == 8) DCI(uint8_t, int64_t);
  else DCI(uint8_t, uint8_t);
#undef DCI
  return mmseg::check_launch("dice_counts_idx");
}

int mmseg_adamw(float* p, const float* g, float* m, float* v, long long n, float lr, float beta1, float beta2,
                float eps, float wd, int step, void* stream) {
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  const float step_size = (float)(lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  const int grid = grid_for(n) > 4096 ? 4096 : grid_for(n);
  const float decay = (float)(1.0 - (double)lr * (double)wd);
  const float omb1 = (float)(1.0 - (double)beta1), omb2 = (float)(1.0 - (double)beta2);
  hipLaunchKernelGGL(adamw_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, p, g, m, v, n, decay, beta1, omb1,
                     beta2, omb2, eps, step_size, bc2s);
  return mmseg::check_launch("adamw");
}

}  // extern "C"
