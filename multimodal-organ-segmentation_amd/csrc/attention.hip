// Multi-head cross-attention of CrossAttentionFusion (reference
// src/models/fusion/attention_fusion.py:77-164) on CDNA4 MFMA.
//
// Every matrix product of the module -- the 1x1 projections (:117-120, :159),
// the scores Q^T K (:147-148), attn . V (:153) and all of their gradients --
// is one batched "NT" GEMM on matrix cores,
//
//     C[b][i][j] (+)= alpha * sum_k A[b][i][k] * B[b][j][k]   (+ bias[j])
//
// with both operands K-contiguous, so every lane's MFMA fragment is one
// 16-byte vector load (8 consecutive k of one row); operands that are not
// K-contiguous are first re-laid out by mmseg_transpose (which also converts
// NCDHW fp32 <-> NDHWC storage dtype at the module boundary).  The batch
// index splits as (outer, inner) = (sample, head) with independent strides, so
// a head is a channel slice of the NDHWC [N][voxels][C] tensors and no
// per-head copies exist.  Softmax (:149) and its backward are one wave per
// row, fp32, fixed-order.  The attention matrix is materialised (N^2 per
// head), which is what the reference computes; the module is only feasible
// at the 12^3 / 6^3 levels, where it is a few MB.
#include "mmseg_common.h"

namespace {

template <typename T>
__device__ __forceinline__ void mfma_acc(f32x4& acc, const V8<T>& a, const V8<T>& b);
template <>
__device__ __forceinline__ void mfma_acc<bf16_t>(f32x4& acc, const V8<bf16_t>& a, const V8<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma_acc<float>(f32x4& acc, const V8<float>& a, const V8<float>& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], acc, 0, 0, 0);
}

struct BgemmArgs {
  const void* a; long long sa_o, sa_i; int lda;
  const void* b; long long sb_o, sb_i; int ldb;
  void* c;       long long sc_o, sc_i; int ldc;
  const float* bias;
  int inner, M, N, K;
  float alpha;
  int accumulate;
};

// Block 256 threads = 2 x 2 waves, block tile 64 x 64, wave tile 32 x 32
// (2 x 2 MFMA tiles of 16 x 16), K step 32; fragments straight from global
// memory (the operands of this module are L2-resident).
template <typename T, typename TO>
__global__ __launch_bounds__(256) void bgemm_nt_kernel(BgemmArgs g) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int tiles_n = (g.N + 63) / 64;
  const int ti = blockIdx.x / tiles_n, tj = blockIdx.x % tiles_n;
  const int bi = blockIdx.y, bo = bi / g.inner, bn = bi % g.inner;
  const T* A = reinterpret_cast<const T*>(g.a) + bo * g.sa_o + bn * g.sa_i;
  const T* B = reinterpret_cast<const T*>(g.b) + bo * g.sb_o + bn * g.sb_i;
  TO* C = reinterpret_cast<TO*>(g.c) + bo * g.sc_o + bn * g.sc_i;
  const int r16 = lane & 15, kg = lane >> 4;
  int arow[2], brow[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    arow[t] = ti * 64 + wm * 32 + t * 16 + r16;
    brow[t] = tj * 64 + wn * 32 + t * 16 + r16;
  }
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < g.K; k0 += 32) {
    const int k = k0 + kg * 8;
    V8<T> af[2], bf[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (arow[t] < g.M && k < g.K) af[t].load(A + (long long)arow[t] * g.lda + k);
      else af[t].zero();
      if (brow[t] < g.N && k < g.K) bf[t].load(B + (long long)brow[t] * g.ldb + k);
      else bf[t].zero();
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) mfma_acc<T>(acc[i][j], af[i], bf[j]);
  }
  // acc[i][j][r] = C[row = ti*64 + wm*32 + i*16 + 4*kg + r][col = tj*64 + wn*32 + j*16 + r16]
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = tj * 64 + wn * 32 + j * 16 + r16;
    if (col >= g.N) continue;
    const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = ti * 64 + wm * 32 + i * 16 + 4 * kg + r;
        if (row >= g.M) continue;
        TO* p = C + (long long)row * g.ldc + col;
        float v = g.alpha * acc[i][j][r] + bv;
        if (g.accumulate) v += (float)*p;
        *p = (TO)v;
      }
  }
}

// dst[b][c][r] = src[b][r][c] with dtype conversion; 32 x 32 tiles through LDS.
template <typename TS, typename TD>
__global__ __launch_bounds__(256) void transpose_kernel(const TS* __restrict__ src, long long s_o, long long s_i,
                                                        int lds_, TD* __restrict__ dst, long long d_o, long long d_i,
                                                        int ldd, int inner, int rows, int cols) {
  __shared__ float tile[32][33];
  const int tiles_c = (cols + 31) / 32;
  const int tr = blockIdx.x / tiles_c, tc = blockIdx.x % tiles_c;
  const int bi = blockIdx.y, bo = bi / inner, bn = bi % inner;
  const TS* S = src + bo * s_o + bn * s_i;
  TD* Dd = dst + bo * d_o + bn * d_i;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = tr * 32 + ty + 8 * k, c = tc * 32 + tx;
    tile[ty + 8 * k][tx] = (r < rows && c < cols) ? (float)S[(long long)r * lds_ + c] : 0.f;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = tc * 32 + ty + 8 * k, r = tr * 32 + tx;
    if (r < rows && c < cols) Dd[(long long)c * ldd + r] = (TD)tile[tx][ty + 8 * k];
  }
}

// P[row][:] = softmax(S[row][:]) (reference attention_fusion.py:149, dim=-1); one wave per row.
template <typename T>
__global__ __launch_bounds__(256) void softmax_rows_kernel(const float* __restrict__ S, int lds_, T* __restrict__ P,
                                                           int ldp, long long rows, int N) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* s = S + row * lds_;
  float mx = -INFINITY;
  for (int m = lane; m < N; m += 64) mx = fmaxf(mx, s[m]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
  for (int m = lane; m < N; m += 64) sum += __expf(s[m] - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  T* p = P + row * ldp;
  for (int m = lane; m < N; m += 64) p[m] = (T)(__expf(s[m] - mx) * inv);
  for (int m = N + lane; m < ldp; m += 64) p[m] = (T)0.f;   // zero row padding (a K pad of the next GEMM)
}

// dS = P * (dP - sum_m dP * P), softmax backward per row.
template <typename T>
__global__ __launch_bounds__(256) void softmax_bwd_rows_kernel(const T* __restrict__ P, int ldp,
                                                               const float* __restrict__ dP, int lddp,
                                                               T* __restrict__ dS, int ldds, long long rows, int N) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const T* p = P + row * ldp;
  const float* d = dP + row * lddp;
  float dot = 0.f;
  for (int m = lane; m < N; m += 64) dot = fmaf((float)p[m], d[m], dot);
  dot = wave_sum(dot);
  T* o = dS + row * ldds;
  for (int m = lane; m < N; m += 64) o[m] = (T)((float)p[m] * (d[m] - dot));
  for (int m = N + lane; m < ldds; m += 64) o[m] = (T)0.f;
}


// ---------------------------------------------------- Swin window attention
// MONAI SwinUNETR WindowAttention (monai/networks/nets/swin_unetr.py, v1.3;
// reference swin_unetr.py:80-96 constructs it): scores + relative-position
// bias B[h][n][m] = table[index[n][m]][h] (+ the shifted-window mask
// M[w][n][m] of window w = b % nw), softmax over m.
__global__ void relpos_bias_kernel(const float* __restrict__ table, const int* __restrict__ index, int heads, int N,
                                   float* __restrict__ bias) {
  const long long total = (long long)heads * N * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const int h = (int)(e / ((long long)N * N));
    const long long nm = e - (long long)h * N * N;
    bias[e] = table[(long long)index[nm] * heads + h];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void softmax_bias_rows_kernel(const float* __restrict__ S, int lds_,
                                                                const float* __restrict__ bias,
                                                                const float* __restrict__ mask, int nw, int heads,
                                                                T* __restrict__ P, int ldp, long long rows, int N) {
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const int n = (int)(row % N);
  const long long bh = row / N;
  const int h = (int)(bh % heads);
  const long long b = bh / heads;
  const float* s = S + row * lds_;
  const float* br = bias ? bias + ((long long)h * N + n) * N : nullptr;
  const float* mr = mask ? mask + ((long long)(b % nw) * N + n) * N : nullptr;
  auto val = [&](int m) {
    float v = s[m];
    if (br) v += br[m];
    if (mr) v += mr[m];
    return v;
  };
  float mx = -INFINITY;
  for (int m = lane; m < N; m += 64) mx = fmaxf(mx, val(m));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  float sum = 0.f;
  for (int m = lane; m < N; m += 64) sum += __expf(val(m) - mx);
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  T* p = P + row * ldp;
  for (int m = lane; m < N; m += 64) p[m] = (T)(__expf(val(m) - mx) * inv);
  for (int m = N + lane; m < ldp; m += 64) p[m] = (T)0.f;
}

// dB[h][n][m] = sum over window-batches b (fixed order) of dS[b][h][n][m]
template <typename T>
__global__ void bias_grad_sum_kernel(const T* __restrict__ dS, int ldn, int B, int heads, int N,
                                     float* __restrict__ dB) {
  const long long hnm = (long long)heads * N * N;
  for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < hnm;
       e += (long long)gridDim.x * blockDim.x) {
    const long long hn = e / N;
    const int m = (int)(e - hn * N);
    float a = 0.f;
    for (int b = 0; b < B; ++b) a += (float)dS[((long long)b * heads * N + hn) * ldn + m];
    dB[e] = a;
  }
}

// gtable[t][h] (+)= sum over the (n, m) pairs with index[n][m] == t (CSR lists).  One wave per (t, h): lanes
// stride over the pair list, then a fixed shuffle tree -> deterministic.  (One thread per entry walked its
// list serially with T*heads = 6.6k threads: 129 us per SwinUNETR stage-0 block at 128^3.)
__global__ __launch_bounds__(256) void relpos_table_grad_kernel(const float* __restrict__ dB,
                                                                const int* __restrict__ offs,
                                                                const int* __restrict__ pairs, int T, int heads,
                                                                int N, float* __restrict__ gtable, int accumulate) {
  const long long total = (long long)T * heads;
  const int lane = threadIdx.x & 63;
  for (long long e = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6; e < total;
       e += ((long long)gridDim.x * blockDim.x) >> 6) {
    const int t = (int)(e / heads), h = (int)(e % heads);
    const float* dh = dB + (long long)h * N * N;
    float a = 0.f;
    for (int k = offs[t] + lane; k < offs[t + 1]; k += 64) a += dh[pairs[k]];
    a = wave_sum(a);
    if (lane == 0) gtable[e] = accumulate ? gtable[e] + a : a;
  }
}
}  // namespace

extern "C" {

int mmseg_bgemm_nt(const void* a, long long sa_outer, long long sa_inner, int lda, const void* b, long long sb_outer,
                   long long sb_inner, int ldb, void* c, long long sc_outer, long long sc_inner, int ldc,
                   const float* bias, int batch, int inner, int M, int N, int K, float alpha, int accumulate,
                   int c_dtype, int dtype, void* stream) {
  MMSEG_REQUIRE(batch >= 1 && inner >= 1 && batch % inner == 0, "bgemm_nt: batch=%d must be a multiple of inner=%d",
                batch, inner);
  // K need not be a multiple of 8: the last 8-element group is read whole, so the caller keeps the row
  // padding [K, round_up(K, 8)) of A or B zero (and the other finite) -- the attention buffers do
  MMSEG_REQUIRE(lda % 8 == 0 && ldb % 8 == 0 && lda >= ((K + 7) & ~7) && ldb >= ((K + 7) & ~7) &&
                    sa_outer % 8 == 0 && sa_inner % 8 == 0 && sb_outer % 8 == 0 && sb_inner % 8 == 0,
                "bgemm_nt: lda, ldb (>= K rounded up to 8) and the A/B batch strides must be multiples of 8");
  MMSEG_REQUIRE(((uintptr_t)a & 15) == 0 && ((uintptr_t)b & 15) == 0, "bgemm_nt: A and B must be 16-B aligned");
  if (M <= 0 || N <= 0) return 0;
  BgemmArgs g{a, sa_outer, sa_inner, lda, b, sb_outer, sb_inner, ldb, c, sc_outer, sc_inner, ldc, bias,
              inner, M, N, K, alpha, accumulate};
  const dim3 grid(ceil_div(M, 64) * ceil_div(N, 64), batch);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MMSEG_BF16) {
    if (c_dtype == MMSEG_BF16) MMSEG_LAUNCH((bgemm_nt_kernel<bf16_t, bf16_t>), grid, dim3(256), 0, s, g);
    else MMSEG_LAUNCH((bgemm_nt_kernel<bf16_t, float>), grid, dim3(256), 0, s, g);
  } else {
    MMSEG_REQUIRE(c_dtype == MMSEG_F32, "bgemm_nt: fp32 operands need an fp32 C");
    MMSEG_LAUNCH((bgemm_nt_kernel<float, float>), grid, dim3(256), 0, s, g);
  }
  mmseg::note_kernel("bgemm_nt_kernel");
  return mmseg::check_launch("bgemm_nt");
}

int mmseg_transpose(const void* src, long long s_outer, long long s_inner, int lds, int src_dtype, void* dst,
                    long long d_outer, long long d_inner, int ldd, int dst_dtype, int batch, int inner, int rows,
                    int cols, void* stream) {
  MMSEG_REQUIRE(batch >= 1 && inner >= 1 && batch % inner == 0, "transpose: batch %% inner != 0");
  if (rows <= 0 || cols <= 0) return 0;
  const dim3 grid(ceil_div(rows, 32) * ceil_div(cols, 32), batch);
  hipStream_t s = (hipStream_t)stream;
#define MMSEG_TR(TS, TD)                                                                                          \
  MMSEG_LAUNCH((transpose_kernel<TS, TD>), grid, dim3(256), 0, s, (const TS*)src, s_outer, s_inner, lds,    \
                     (TD*)dst, d_outer, d_inner, ldd, inner, rows, cols)
  if (src_dtype == MMSEG_F32 && dst_dtype == MMSEG_F32) MMSEG_TR(float, float);
  else if (src_dtype == MMSEG_F32) MMSEG_TR(float, bf16_t);
  else if (dst_dtype == MMSEG_F32) MMSEG_TR(bf16_t, float);
  else MMSEG_TR(bf16_t, bf16_t);
#undef MMSEG_TR
  return mmseg::check_launch("transpose");
}

int mmseg_softmax_rows(const float* S, int lds, void* P, int ldp, long long rows, int N, int dtype, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(softmax_rows_kernel<bf16_t>, grid, dim3(256), 0, s, S, lds, (bf16_t*)P, ldp, rows, N);
  else
    MMSEG_LAUNCH(softmax_rows_kernel<float>, grid, dim3(256), 0, s, S, lds, (float*)P, ldp, rows, N);
  return mmseg::check_launch("softmax_rows");
}

int mmseg_softmax_bwd_rows(const void* P, int ldp, const float* dP, int lddp, void* dS, int ldds, long long rows,
                           int N, int dtype, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(softmax_bwd_rows_kernel<bf16_t>, grid, dim3(256), 0, s, (const bf16_t*)P, ldp, dP, lddp,
                       (bf16_t*)dS, ldds, rows, N);
  else
    MMSEG_LAUNCH(softmax_bwd_rows_kernel<float>, grid, dim3(256), 0, s, (const float*)P, ldp, dP, lddp,
                       (float*)dS, ldds, rows, N);
  return mmseg::check_launch("softmax_bwd_rows");
}

int mmseg_relpos_bias(const float* table, const int* index, int heads, int N, float* bias, void* stream) {
  const long long total = (long long)heads * N * N;
  MMSEG_LAUNCH(relpos_bias_kernel, dim3((unsigned)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192)),
                     dim3(256), 0, (hipStream_t)stream, table, index, heads, N, bias);
  return mmseg::check_launch("relpos_bias");
}

int mmseg_softmax_bias_rows(const float* S, int lds, const float* bias, const float* mask, int nw, int heads, void* P,
                            int ldp, long long rows, int N, int dtype, void* stream) {
  MMSEG_REQUIRE(!mask || nw >= 1, "softmax_bias_rows: mask needs nw >= 1");
  MMSEG_REQUIRE(rows % ((long long)N * heads) == 0, "softmax_bias_rows: rows must be windows x heads x N");
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)((rows + 3) / 4));
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(softmax_bias_rows_kernel<bf16_t>, grid, dim3(256), 0, s, S, lds, bias, mask, nw, heads,
                       (bf16_t*)P, ldp, rows, N);
  else
    MMSEG_LAUNCH(softmax_bias_rows_kernel<float>, grid, dim3(256), 0, s, S, lds, bias, mask, nw, heads,
                       (float*)P, ldp, rows, N);
  return mmseg::check_launch("softmax_bias_rows");
}

int mmseg_relpos_table_grad(const void* dS, int ldn, int B, int heads, int N, float* dB, const int* offs,
                            const int* pairs, int T, float* gtable, int accumulate, int dtype, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long long hnm = (long long)heads * N * N;
  const unsigned g1 = (unsigned)((hnm + 255) / 256 < 8192 ? (hnm + 255) / 256 : 8192);
  if (dtype == MMSEG_BF16)
    MMSEG_LAUNCH(bias_grad_sum_kernel<bf16_t>, dim3(g1), dim3(256), 0, s, (const bf16_t*)dS, ldn, B, heads, N,
                       dB);
  else
    MMSEG_LAUNCH(bias_grad_sum_kernel<float>, dim3(g1), dim3(256), 0, s, (const float*)dS, ldn, B, heads, N,
                       dB);
  if (mmseg::check_launch("bias_grad_sum")) return 1;
  const long long th = (long long)T * heads;
  MMSEG_LAUNCH(relpos_table_grad_kernel, dim3((unsigned)std::min<long long>((th + 3) / 4, 8192)), dim3(256), 0, s,
                     dB, offs, pairs, T,
                     heads, N, gtable, accumulate);
  return mmseg::check_launch("relpos_table_grad");
}

}  // extern "C"
