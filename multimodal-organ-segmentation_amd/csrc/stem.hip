// First 3^3 convolution of each encoder ("stem"): Conv3d(Cr -> Co, k3, p1)
// with Cr = 1 (one modality per DualEncoder encoder, dual_encoder.py:66-70)
// or 2-3 (early-fusion UNet3D, unet.py:154-157).
//
// The generic kernels see the stem as a Cin = 8 conv (the input is packed as
// 8-channel NDHWC tiles) and therefore do 8/Cr times the needed MACs.  Here
// K = 27*Cr taps*channels exactly (padded to KP, a multiple of 32):
//   stem_fwd   : y[v][co] = b[co] + sum_k im2col[v][k] * w[co][k]
//   stem_wgrad : dW[co][k] = sum_v dy[v][co] * im2col[v][k]  (+ db[co] = sum_v dy[v][co])
// im2col is never materialised: a block stages the 6x10x10 input halo of its
// 4x8x8 output brick in LDS and every lane gathers its MFMA fragment from it.
// Weights are read straight from the fp32 master copy (no packed image).
#include "mmseg_common.h"

namespace {

constexpr int SZ = 4, SY = 8, SX = 8;                 // output brick (256 voxels)
constexpr int SHZ = SZ + 2, SHY = SY + 2, SHX = SX + 2;
constexpr int SHV = SHZ * SHY * SHX;                  // 600 halo voxels
constexpr int SCR = 8;                                 // packed input channels per voxel

template <typename T>
__device__ __forceinline__ void stem_mfma(f32x4& acc, const V8<T>& a, const V8<T>& b);
template <>
__device__ __forceinline__ void stem_mfma<bf16_t>(f32x4& acc, const V8<bf16_t>& a, const V8<bf16_t>& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void stem_mfma<float>(f32x4& acc, const V8<float>& a, const V8<float>& b) {
#pragma unroll
  for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], acc, 0, 0, 0);
}

// halo voxel of brick voxel r (z = r>>6, y = (r>>3)&7, x = r&7) shifted by tap t
__device__ __forceinline__ int stem_hv(int r, int t) {
  const int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;
  return (((r >> 6) + kz) * SHY + ((r >> 3) & 7) + ky) * SHX + (r & 7) + kx;
}

struct StemArgs {
  const void* x; int ldx; int cr;       // packed input, real channels
  const float* w; const float* bias;    // [Co][cr][27], [Co]
  void* y; int ldy;
  const void* dy; int lddy;             // wgrad
  float* part; float* bias_part;        // wgrad partials [ks][Co][KP], [ks][Co]
  int N, D, H, W, Co, KP;
  int ksplit;
};

template <typename T>
__device__ __forceinline__ void stem_stage_halo(const StemArgs& g, T* Hl, long long nbase, int z0, int y0, int x0) {
  const T* X = reinterpret_cast<const T*>(g.x);
  const long long HW = (long long)g.H * g.W;
  for (int h = threadIdx.x; h < SHV; h += blockDim.x) {
    const int hx = h % SHX, hy = (h / SHX) % SHY, hz = h / (SHX * SHY);
    const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
    V8<T> v;
    if ((unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W) {
      const T* src = X + (nbase + z * HW + (long long)y * g.W + x) * g.ldx;
      if (g.ldx == SCR) {
        v.load(src);
      } else {   // compact input (ldx = cr): only the real channels cross HBM
        v.zero();
        for (int c = 0; c < g.cr; ++c) v.set(c, (float)src[c]);
      }
    } else {
      v.zero();
    }
    v.store(Hl + h * SCR);
  }
}

// ---------------------------------------------------------------- forward
// block = one 4x8x8 brick x all Co (<= 64) columns; wave w owns brick z-slice w
// (4 row tiles of 16 voxels)
template <typename T, int RN>
__global__ __launch_bounds__(256) void stem_fwd_kernel(StemArgs g) {
  // dynamic LDS: halo [600][8] | weights [Co][KP+8]; the epilogue tile [256][Co+8] reuses it after the MFMAs
  extern __shared__ __attribute__((aligned(16))) unsigned char stem_lds[];
  T* Hl = reinterpret_cast<T*>(stem_lds);
  T* Wl = Hl + SHV * SCR;
  T* El = Hl;
  const int WP = g.KP + 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / SZ, by_n = g.H / SY, bx_n = g.W / SX;
  int b = blockIdx.x;
  const int bx = b % bx_n; b /= bx_n;
  const int by = b % by_n; b /= by_n;
  const int bz = b % bz_n;
  const int n = b / bz_n;
  const long long HW = (long long)g.H * g.W;
  const long long nbase = (long long)n * g.D * HW;
  const int z0 = bz * SZ, y0 = by * SY, x0 = bx * SX;
  const int K = 27 * g.cr;
  stem_stage_halo<T>(g, Hl, nbase, z0, y0, x0);
  for (int e = tid; e < g.Co * g.KP; e += 256) {
    const int co = e / g.KP, k = e - co * g.KP;
    float v = 0.f;
    if (k < K) {
      const int t = k / g.cr, c = k - t * g.cr;
      v = g.w[((long long)co * g.cr + c) * 27 + t];
    }
    Wl[co * WP + k] = from_f<T>(v);
  }
  __syncthreads();
  const int r16 = lane & 15, kg = lane >> 4;
  f32x4 acc[4][RN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int rbase[4];   // halo index (tap 0) of the lane's row in each row tile
#pragma unroll
  for (int i = 0; i < 4; ++i) rbase[i] = stem_hv(wave * 64 + i * 16 + r16, 0);
  for (int kb = 0; kb < g.KP; kb += 32) {
    // this lane's 8 im2col columns: LDS element offset (tap shift * 8 + channel), -1 = padding
    int koff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = kb + kg * 8 + j;
      const int t = k / g.cr, c = k - t * g.cr;
      koff[j] = k < K ? stem_hv(0, t) * SCR + c : -1;
    }
    V8<T> af[4], bf[RN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) af[i].set(j, koff[j] >= 0 ? (float)Hl[rbase[i] * SCR + koff[j]] : 0.f);
#pragma unroll
    for (int j = 0; j < RN; ++j) bf[j].load(Wl + (j * 16 + r16) * WP + kb + kg * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) stem_mfma<T>(acc[i][j], af[i], bf[j]);
  }
  constexpr int EP = RN * 16 + 8;
  __syncthreads();   // El aliases the halo / weights
#pragma unroll
  for (int j = 0; j < RN; ++j) {
    const int col = j * 16 + r16;
    const float bv = g.bias ? g.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) El[(wave * 64 + i * 16 + kg * 4 + r) * EP + col] = from_f<T>(acc[i][j][r] + bv);
  }
  __syncthreads();
  T* Y = reinterpret_cast<T*>(g.y);
  constexpr int CG = RN * 2;
  for (int e = tid; e < 256 * CG; e += 256) {
    const int v = e / CG, cg = e % CG;
    const int z = z0 + (v >> 6), y = y0 + ((v >> 3) & 7), x = x0 + (v & 7);
    V8<T> o;
    o.load(El + v * EP + cg * 8);
    o.store(Y + (nbase + z * HW + (long long)y * g.W + x) * g.ldy + cg * 8);
  }
}

// ------------------------------------------------------------ weight grad
// block = a contiguous range of bricks; wave w accumulates the brick's voxel
// steps w, w+4 (2 x 32 voxels) into the full [Co][KP] tile; the 4 wave tiles
// are added in order at the end (deterministic).
template <typename T, int RM, int RNK>
__global__ __launch_bounds__(256) void stem_wgrad_kernel(StemArgs g) {
  constexpr int DP = RM * 16 + 8;
  constexpr int HB = SHV * SCR * sizeof(T), DB = 256 * DP * sizeof(T);
  constexpr int RB = 4 * RM * 16 * (RNK * 16 + 1) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[(HB + DB) > RB ? (HB + DB) : RB];
  T* Hl = reinterpret_cast<T*>(lds_raw);
  T* Dl = reinterpret_cast<T*>(lds_raw + HB);
  float (*red)[RM * 16][RNK * 16 + 1] = reinterpret_cast<float (*)[RM * 16][RNK * 16 + 1]>(lds_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / SZ, by_n = g.H / SY, bx_n = g.W / SX;
  const long long nbrick = (long long)g.N * bz_n * by_n * bx_n;
  const long long bpk = (nbrick + g.ksplit - 1) / g.ksplit;
  const long long b0 = blockIdx.x * bpk;
  const long long b1 = b0 + bpk < nbrick ? b0 + bpk : nbrick;
  const long long HW = (long long)g.H * g.W;
  const int K = 27 * g.cr;
  const T* Dy = reinterpret_cast<const T*>(g.dy);
  const int r16 = lane & 15, kg = lane >> 4;
  f32x4 acc[RM][RNK];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RNK; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;   // bias partial of channel tid % Co over voxel slice tid / Co
  int bko[RNK];       // this lane's im2col column per k tile: LDS offset (tap shift * 8 + channel), -1 = padding
#pragma unroll
  for (int jt = 0; jt < RNK; ++jt) {
    const int k = jt * 16 + r16;
    const int t = k / g.cr, c = k - t * g.cr;
    bko[jt] = k < K ? stem_hv(0, t) * SCR + c : -1;
  }
  for (long long b = b0; b < b1; ++b) {
    long long q = b;
    const int bx = (int)(q % bx_n); q /= bx_n;
    const int by = (int)(q % by_n); q /= by_n;
    const int bz = (int)(q % bz_n);
    const long long nbase = (q / bz_n) * g.D * HW;
    const int z0 = bz * SZ, y0 = by * SY, x0 = bx * SX;
    __syncthreads();   // previous brick fully consumed
    stem_stage_halo<T>(g, Hl, nbase, z0, y0, x0);
    const int CGd = g.Co / 8;
    for (int e = tid; e < 256 * CGd; e += 256) {
      const int v = e / CGd, cg = e % CGd;
      const int z = z0 + (v >> 6), y = y0 + ((v >> 3) & 7), x = x0 + (v & 7);
      V8<T> d;
      d.load(Dy + (nbase + z * HW + (long long)y * g.W + x) * g.lddy + cg * 8);
      d.store(Dl + v * DP + cg * 8);
    }
    __syncthreads();
    if (g.bias_part) {   // thread = (channel tid % Co, voxel slice tid / Co)
      const int c = tid % g.Co, nsl = 256 / g.Co;
      for (int v = tid / g.Co; v < 256; v += nsl) bsum += (float)Dl[v * DP + c];
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int vb = (wave + 4 * s) * 32;       // voxel step
      // A = dy^T: row co, k = voxels vb + 8*kg + j
      V8<T> af[RM], bf[RNK];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) af[i].set(j, (float)Dl[(vb + kg * 8 + j) * DP + i * 16 + r16]);
      // B = im2col: column k = jt*16 + r16, k-dim = the same 8 voxels (one x-row: halo j + const)
      const int hb = stem_hv(vb + kg * 8, 0) * SCR;
#pragma unroll
      for (int jt = 0; jt < RNK; ++jt) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
          bf[jt].set(j, bko[jt] >= 0 ? (float)Hl[hb + j * SCR + bko[jt]] : 0.f);
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jt = 0; jt < RNK; ++jt) stem_mfma<T>(acc[i][jt], af[i], bf[jt]);
    }
  }
  // fixed-order combine of the 4 wave tiles -> part[ks][Co][KP] (red aliases the stage buffers)
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jt = 0; jt < RNK; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][i * 16 + kg * 4 + r][jt * 16 + r16] = acc[i][jt][r];
  __syncthreads();
  for (int e = tid; e < g.Co * g.KP; e += 256) {
    const int co = e / g.KP, k = e - co * g.KP;
    const float v = ((red[0][co][k] + red[1][co][k]) + red[2][co][k]) + red[3][co][k];
    g.part[((long long)blockIdx.x * g.Co + co) * g.KP + k] = v;
  }
  if (g.bias_part) {
    __syncthreads();
    float* rb = reinterpret_cast<float*>(lds_raw);
    rb[tid] = bsum;
    __syncthreads();
    if (tid < g.Co) {
      float a = 0.f;
      for (int sl = 0; sl < 256 / g.Co; ++sl) a += rb[sl * g.Co + tid];
      g.bias_part[(long long)blockIdx.x * g.Co + tid] = a;
    }
  }
}

int stem_kp(int cr) { return ((27 * cr + 31) / 32) * 32; }

}  // namespace

extern "C" {

int mmseg_stem_ok(int cr, int Co, int D, int H, int W, int ldx, int ldy) {
  return cr >= 1 && cr <= 4 && (ldx == SCR || ldx == cr) && (Co == 16 || Co == 32) && ldy % 8 == 0 && D % SZ == 0 &&
         H % SY == 0 && W % SX == 0;
}

int mmseg_stem_fwd(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N, int D,
                   int H, int W, int Co, int dtype, void* stream) {
  MMSEG_REQUIRE(mmseg_stem_ok(cr, Co, D, H, W, ldx, ldy), "stem_fwd: unsupported shape (cr=%d Co=%d %dx%dx%d)", cr,
                Co, D, H, W);
  StemArgs g{x, ldx, cr, w, bias, y, ldy, nullptr, 0, nullptr, nullptr, N, D, H, W, Co, stem_kp(cr), 1};
  const dim3 grid(N * (D / SZ) * (H / SY) * (W / SX));
  hipStream_t s = (hipStream_t)stream;
  mmseg::note_kernel("stem_fwd_kernel");
  const size_t ts = dtype == MMSEG_BF16 ? 2 : 4;
  const size_t stage = (size_t)(SHV * SCR + Co * (stem_kp(cr) + 8)) * ts, epi = (size_t)256 * (Co + 8) * ts;
  const size_t shm = stage > epi ? stage : epi;
  if (dtype == MMSEG_BF16) {
    if (Co == 16) hipLaunchKernelGGL((stem_fwd_kernel<bf16_t, 1>), grid, dim3(256), shm, s, g);
    else hipLaunchKernelGGL((stem_fwd_kernel<bf16_t, 2>), grid, dim3(256), shm, s, g);
  } else {
    if (Co == 16) hipLaunchKernelGGL((stem_fwd_kernel<float, 1>), grid, dim3(256), shm, s, g);
    else hipLaunchKernelGGL((stem_fwd_kernel<float, 2>), grid, dim3(256), shm, s, g);
  }
  return mmseg::check_launch("stem_fwd");
}

// K columns of the stem weight-gradient partials (27*cr padded to 32).
int mmseg_stem_kp(int cr) { return stem_kp(cr); }

int mmseg_stem_wgrad_splits(int N, int D, int H, int W, int want) {
  const long long nbrick = (long long)N * (D / SZ) * (H / SY) * (W / SX);
  long long ks = want < nbrick ? want : nbrick;
  if (ks < 1) ks = 1;
  const long long bpk = (nbrick + ks - 1) / ks;
  return (int)((nbrick + bpk - 1) / bpk);
}

// part[ks][Co][KP] (+ bias_part[ks][Co]); reduce with mmseg_wgrad_reduce(Ca=Co, Ncols=KP, cpad=cr, creal=cr, ntap=27)
int mmseg_stem_wgrad(const void* dy, int lddy, const void* x, int ldx, int cr, float* part, float* bias_part, int N,
                     int D, int H, int W, int Co, int ksplit, int dtype, void* stream) {
  MMSEG_REQUIRE(mmseg_stem_ok(cr, Co, D, H, W, ldx, lddy), "stem_wgrad: unsupported shape");
  StemArgs g{x, ldx, cr, nullptr, nullptr, nullptr, 0, dy, lddy, part, bias_part, N, D, H, W, Co, stem_kp(cr),
             ksplit};
  hipStream_t s = (hipStream_t)stream;
  mmseg::note_kernel("stem_wgrad_kernel");
  const dim3 grid(ksplit), blk(256);
  const int rnk = stem_kp(cr) / 16;   // 2, 4, 6, 8
#define STEM_WG(TT, RM_)                                                                   \
  switch (rnk) {                                                                           \
    case 2: hipLaunchKernelGGL((stem_wgrad_kernel<TT, RM_, 2>), grid, blk, 0, s, g); break; \
    case 4: hipLaunchKernelGGL((stem_wgrad_kernel<TT, RM_, 4>), grid, blk, 0, s, g); break; \
    case 6: hipLaunchKernelGGL((stem_wgrad_kernel<TT, RM_, 6>), grid, blk, 0, s, g); break; \
    default: hipLaunchKernelGGL((stem_wgrad_kernel<TT, RM_, 8>), grid, blk, 0, s, g); break; \
  }
  if (dtype == MMSEG_BF16) {
    if (Co == 16) { STEM_WG(bf16_t, 1) } else { STEM_WG(bf16_t, 2) }
  } else {
    if (Co == 16) { STEM_WG(float, 1) } else { STEM_WG(float, 2) }
  }
#undef STEM_WG
  return mmseg::check_launch("stem_wgrad");
}

}  // extern "C"
