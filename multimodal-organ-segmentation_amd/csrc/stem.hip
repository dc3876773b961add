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

#include <type_traits>

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
  // wgrad with the InstanceNorm + ReLU backward applied on staging (mmseg_stem_wgrad_inb): dy is the gradient of
  // the norm's OUTPUT, inx its pre-norm input (pitch ldinx), inmean / inrstd [N][Co] its statistics and incoef
  // [N][Co][2] the finalised (mean g, mean g xhat); the staged value is in_bwd_apply's
  // rstd (g - a - xhat b), g = dy [xhat > 0], rounded to T, so the norm's input gradient is never written
  const void* inx; int ldinx;
  const float* inmean; const float* inrstd; const float* incoef;
  // forward: per-brick InstanceNorm partials of the stored output, [brick][Co][2] = (mean, M2) over its 256 voxels
  // (the layout of conv_gemm.hip brick_in_stats; merged by mmseg_instnorm_stats_bricks), or null
  float* stats;
};

// Halo of a brick in LDS, compact: [600 halo voxels][CR channels] (the padded 8-channel input layout would
// put 16 B between the 2-B values one lane gathers, a 4-way bank conflict on every gather, r02 PMC).
template <typename T, int CR>
__device__ __forceinline__ void stem_stage_halo(const StemArgs& g, T* Hl, long long nbase, int z0, int y0, int x0) {
  const T* X = reinterpret_cast<const T*>(g.x);
  const long long HW = (long long)g.H * g.W;
  for (int h = threadIdx.x; h < SHV; h += blockDim.x) {
    const int hx = h % SHX, hy = (h / SHX) % SHY, hz = h / (SHX * SHY);
    const int z = z0 - 1 + hz, y = y0 - 1 + hy, x = x0 - 1 + hx;
    const bool in = (unsigned)z < (unsigned)g.D && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
    const T* src = X + (nbase + z * HW + (long long)y * g.W + x) * g.ldx;
#pragma unroll
    for (int c = 0; c < CR; ++c) Hl[h * CR + c] = in ? src[c] : (T)0.f;
  }
}

// im2col column k of the stem (k = tap * CR + channel, 27 CR real columns padded to KP): its offset in the
// compact halo relative to the row's tap-0 voxel, -1 for padding.  Built once per block into LDS.
template <int CR>
__device__ __forceinline__ int stem_koff(int k) {
  const int t = k / CR, c = k - t * CR;
  return k < 27 * CR ? stem_hv(0, t) * CR + c : -1;
}

// ---------------------------------------------------------------- forward
// block = one 4x8x8 brick x all CO (16 / 32) columns; wave w owns brick z-slice w (4 row tiles of 16 voxels).
// CR and CO are compile-time: the runtime divisions by cr / KP in the column bookkeeping were most of the
// kernel's VALU instructions (1,056 per wave for 8 MFMAs, r02 PMC).
template <typename T, int RN, int CR>
__global__ __launch_bounds__(256) void stem_fwd_kernel(StemArgs g) {
  constexpr int K = 27 * CR, KP = ((K + 31) / 32) * 32, WP = KP + 8, CO = RN * 16, EP = CO + 8;
  constexpr int HB = ((SHV * CR * (int)sizeof(T) + 15) / 16) * 16;
  constexpr int WB = CO * WP * (int)sizeof(T);
  constexpr int KB = KP * 4;
  constexpr int EB = 256 * EP * (int)sizeof(T);
  constexpr int LB = (HB + WB + KB) > EB ? (HB + WB + KB) : EB;
  __shared__ __attribute__((aligned(16))) unsigned char lds[LB];
  T* Hl = reinterpret_cast<T*>(lds);
  T* Wl = reinterpret_cast<T*>(lds + HB);
  int* Kl = reinterpret_cast<int*>(lds + HB + WB);
  T* El = reinterpret_cast<T*>(lds);   // epilogue tile, after the MFMAs
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
  stem_stage_halo<T, CR>(g, Hl, nbase, z0, y0, x0);
  for (int e = tid; e < CO * KP; e += 256) {
    const int co = e / KP, k = e - co * KP;
    const int t = k / CR, c = k - t * CR;
    Wl[co * WP + k] = from_f<T>(k < K ? g.w[(co * CR + c) * 27 + t] : 0.f);
  }
  if (tid < KP) Kl[tid] = stem_koff<CR>(tid);
  __syncthreads();
  const int r16 = lane & 15, kg = lane >> 4;
  f32x4 acc[4][RN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  int rbase[4];   // compact-halo offset (tap 0) of the lane's row in each row tile
#pragma unroll
  for (int i = 0; i < 4; ++i) rbase[i] = stem_hv(wave * 64 + i * 16 + r16, 0) * CR;
#pragma unroll
  for (int kb = 0; kb < KP; kb += 32) {
    int koff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) koff[j] = Kl[kb + kg * 8 + j];
    V8<T> af[4], bf[RN];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) af[i].v[j] = koff[j] >= 0 ? Hl[rbase[i] + koff[j]] : (T)0.f;
#pragma unroll
    for (int j = 0; j < RN; ++j) bf[j].load(Wl + (j * 16 + r16) * WP + kb + kg * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < RN; ++j) stem_mfma<T>(acc[i][j], af[i], bf[j]);
  }
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
  // stats: Welford over the thread's CG voxels of its channel group tid % CG (the values as stored)
  float smu[8], sm2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) smu[j] = sm2[j] = 0.f;
#pragma unroll
  for (int q = 0; q < CG; ++q) {
    const int e = tid + q * 256;
    const int v = e / CG, cg = e % CG;
    const int z = z0 + (v >> 6), y = y0 + ((v >> 3) & 7), x = x0 + (v & 7);
    V8<T> o;
    o.load(El + v * EP + cg * 8);
    o.store(Y + (nbase + z * HW + (long long)y * g.W + x) * g.ldy + cg * 8);
    if (g.stats) {
      const float inv = 1.f / (float)(q + 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = o.get(j), d = xv - smu[j];
        smu[j] = fmaf(d, inv, smu[j]);
        sm2[j] = fmaf(d, xv - smu[j], sm2[j]);
      }
    }
  }
  if (g.stats) {
    // equal-count Chan merges, fixed order, over the lanes of a wave holding the same channel group (xor CG .. 32,
    // count per lane CG << level); each wave writes the partial of its brick z-slice (64 voxels), so the block
    // needs no barrier or serial merge (a block-level merge made the kernel 16 us slower at 96^3 B=2)
    float cnt = (float)CG;
#pragma unroll
    for (int o = CG; o < 64; o <<= 1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float mb = __shfl_xor(smu[j], o, 64), m2b = __shfl_xor(sm2[j], o, 64);
        const bool lo = (lane & o) == 0;   // both partners form the same value
        const float m1 = lo ? smu[j] : mb, m2 = lo ? mb : smu[j];
        const float d = m2 - m1;
        sm2[j] = (lo ? sm2[j] + m2b : m2b + sm2[j]) + d * d * (0.5f * cnt);
        smu[j] = m1 + 0.5f * d;
      }
      cnt *= 2.f;
    }
    if (lane < CG) {
      float* out = g.stats + (((long long)blockIdx.x * 4 + wave) * CO + lane * 8) * 2;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        out[2 * j] = smu[j];
        out[2 * j + 1] = sm2[j];
      }
    }
  }
}

// ------------------------------------------------------------ weight grad
// block = a contiguous range of bricks; wave w accumulates the brick's voxel
// steps w, w+4 (2 x 32 voxels) into the full [CO][KP] tile; the 4 wave tiles
// are added in order at the end (deterministic).
// CR = 1 (the DualEncoder stems): held to 128 VGPRs, 4 waves / SIMD, so all 1,024 blocks of the 96^3 B=2 grid
// are resident at once (at 3 waves / SIMD the last 256 ran as a second round); wider CR would spill.
template <typename T, int RM, int RNK, int CR, bool INB = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(CR == 1 ? 4 : 1))) void stem_wgrad_kernel(StemArgs g) {
  constexpr int K = 27 * CR, KP = RNK * 16, CO = RM * 16, CGd = CO / 8;
  static_assert(KP == ((K + 31) / 32) * 32, "KP = 27 CR padded to 32");
  constexpr int DP = CO + 8;
  constexpr int HB = ((SHV * CR * (int)sizeof(T) + 15) / 16) * 16, DB = 256 * DP * (int)sizeof(T);
  constexpr int RB = 4 * CO * (KP + 1) * 4;
  constexpr int SB = INB ? CO * 16 : 0;   // INB: the sample's norm statistics [CO] x (mean, rstd, a, b)
  constexpr int LB = (HB + DB + KP * 4 + SB) > RB ? (HB + DB + KP * 4 + SB) : RB;
  __shared__ __attribute__((aligned(16))) unsigned char lds_raw[LB];
  T* Hl = reinterpret_cast<T*>(lds_raw);
  T* Dl = reinterpret_cast<T*>(lds_raw + HB);
  int* Kl = reinterpret_cast<int*>(lds_raw + HB + DB);
  float4* Sl = reinterpret_cast<float4*>(lds_raw + HB + DB + KP * 4);
  float (*red)[CO][KP + 1] = reinterpret_cast<float (*)[CO][KP + 1]>(lds_raw);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int bz_n = g.D / SZ, by_n = g.H / SY, bx_n = g.W / SX;
  const int nbrick = g.N * bz_n * by_n * bx_n;
  const int bpk = (nbrick + g.ksplit - 1) / g.ksplit;
  const int b0 = blockIdx.x * bpk;
  const int b1 = b0 + bpk < nbrick ? b0 + bpk : nbrick;
  const long long HW = (long long)g.H * g.W;
  const T* Dy = reinterpret_cast<const T*>(g.dy);
  const int r16 = lane & 15, kg = lane >> 4;
  if (tid < KP) Kl[tid] = stem_koff<CR>(tid);
  f32x4 acc[RM][RNK];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RNK; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;   // bias partial of channel tid % CO over voxel slice tid / CO
  int bko[RNK];       // this lane's im2col column per k tile (compact-halo offset), -1 = padding
  // INB: the statistics of the current sample live in LDS (Sl), read per channel while staging -- in registers
  // (32 VGPRs) they held the kernel at 3 waves / SIMD, 768 resident blocks for the 1,024-split grid
  int in_n = -1;
  // dy (and, INB, the norm's pre-norm input) of the NEXT brick is loaded into registers before this brick's MFMA
  // phase, so its HBM latency hides behind the MFMAs (thread item qq: voxel (tid + 256 qq) / CGd, channel group
  // tid % CGd)
  V8<T> pd[CGd], px[INB ? CGd : 1];
  auto prefetch = [&](int b) {
    int q = b;
    const int bx = q % bx_n; q /= bx_n;
    const int by = q % by_n; q /= by_n;
    const int bz = q % bz_n;
    const long long nb = (long long)(q / bz_n) * g.D * HW;
    const int z0 = bz * SZ, y0 = by * SY, x0 = bx * SX;
#pragma unroll
    for (int qq = 0; qq < CGd; ++qq) {
      const int e = tid + qq * 256;
      const int v = e / CGd, cg = e % CGd;
      const int z = z0 + (v >> 6), y = y0 + ((v >> 3) & 7), x = x0 + (v & 7);
      const long long vox = nb + z * HW + (long long)y * g.W + x;
      pd[qq].load(Dy + vox * g.lddy + cg * 8);
      if constexpr (INB) px[qq].load(reinterpret_cast<const T*>(g.inx) + vox * g.ldinx + cg * 8);
    }
  };
  if (b0 < b1) prefetch(b0);
  for (int b = b0; b < b1; ++b) {
    int q = b;
    const int bx = q % bx_n; q /= bx_n;
    const int by = q % by_n; q /= by_n;
    const int bz = q % bz_n;
    const long long nbase = (long long)(q / bz_n) * g.D * HW;
    const int z0 = bz * SZ, y0 = by * SY, x0 = bx * SX;
    if constexpr (INB) {
      // (the previous brick's staging read Sl before its second barrier)
      const int n = q / bz_n;
      if (n != in_n) {
        in_n = n;
        if (tid < CO) {
          const int c = n * CO + tid;
          Sl[tid] = make_float4(g.inmean[c], g.inrstd[c], g.incoef[c * 2], g.incoef[c * 2 + 1]);
        }
      }
    }
    __syncthreads();   // previous brick fully consumed (and, first time round, Kl written)
    if (b == b0) {
#pragma unroll
      for (int jt = 0; jt < RNK; ++jt) bko[jt] = Kl[jt * 16 + r16];
    }
    stem_stage_halo<T, CR>(g, Hl, nbase, z0, y0, x0);
#pragma unroll
    for (int qq = 0; qq < CGd; ++qq) {
      const int e = tid + qq * 256;
      const int v = e / CGd, cg = e % CGd;
      V8<T> d = pd[qq];
      if constexpr (INB) {   // in_bwd_apply's operations (DyCtx with p1 = dy, scale 1, no beta / pool)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float4 st = Sl[cg * 8 + j];   // (mean, rstd, a, b)
          const float dyv = d.get(j) * 1.f + 0.f;
          const float h = (px[qq].get(j) - st.x) * st.y;
          const float gg = h > 0.f ? dyv : 0.f;
          d.set(j, st.y * (gg - st.z - h * st.w));
        }
      }
      d.store(Dl + v * DP + cg * 8);
    }
    if (b + 1 < b1) prefetch(b + 1);
    __syncthreads();
    if (g.bias_part) {   // thread = (channel tid % CO, voxel slice tid / CO)
      const int c = tid % CO;
      for (int v = tid / CO; v < 256; v += 256 / CO) bsum += (float)Dl[v * DP + c];
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int vb = (wave + 4 * s) * 32;       // voxel step
      // A = dy^T: row co, k = voxels vb + 8*kg + j
      V8<T> af[RM], bf[RNK];
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) af[i].v[j] = Dl[(vb + kg * 8 + j) * DP + i * 16 + r16];
      // B = im2col: column k = jt*16 + r16, k-dim = the same 8 voxels (one x-row: halo j + const)
      const int hb = stem_hv(vb + kg * 8, 0) * CR;
#pragma unroll
      for (int jt = 0; jt < RNK; ++jt) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bf[jt].v[j] = bko[jt] >= 0 ? Hl[hb + j * CR + bko[jt]] : (T)0.f;
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jt = 0; jt < RNK; ++jt) stem_mfma<T>(acc[i][jt], af[i], bf[jt]);
    }
  }
  // fixed-order combine of the 4 wave tiles -> part[ks][CO][KP] (red aliases the stage buffers)
  __syncthreads();
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int jt = 0; jt < RNK; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][i * 16 + kg * 4 + r][jt * 16 + r16] = acc[i][jt][r];
  __syncthreads();
  for (int e = tid; e < CO * KP; e += 256) {
    const int co = e / KP, k = e - co * KP;
    const float v = ((red[0][co][k] + red[1][co][k]) + red[2][co][k]) + red[3][co][k];
    g.part[((long long)blockIdx.x * CO + co) * KP + k] = v;
  }
  if (g.bias_part) {
    __syncthreads();
    float* rb = reinterpret_cast<float*>(lds_raw);
    rb[tid] = bsum;
    __syncthreads();
    if (tid < CO) {
      float a = 0.f;
      for (int sl = 0; sl < 256 / CO; ++sl) a += rb[sl * CO + tid];
      g.bias_part[(long long)blockIdx.x * CO + tid] = a;
    }
  }
}

int stem_kp(int cr) { return ((27 * cr + 31) / 32) * 32; }

}  // namespace

extern "C" {

int mmseg_stem_ok(int cr, int Co, int D, int H, int W, int ldx, int ldy) {
  // Co 48: SwinUNETR's encoder1 conv1 (2 -> 48 at 128^3), no bias, no fused statistics
  return cr >= 1 && cr <= 4 && (ldx == SCR || ldx == cr) && (Co == 16 || Co == 32 || Co == 48) && ldy % 8 == 0 &&
         D % SZ == 0 && H % SY == 0 && W % SX == 0;
}

int mmseg_stem_fwd_stats(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N,
                         int D, int H, int W, int Co, float* stats, int dtype, void* stream);

int mmseg_stem_fwd(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N, int D,
                   int H, int W, int Co, int dtype, void* stream) {
  return mmseg_stem_fwd_stats(x, ldx, cr, w, bias, y, ldy, N, D, H, W, Co, nullptr, dtype, stream);
}

// Partials per sample of the stem forward's fused InstanceNorm statistics: one per z-slice of each 4x8x8 brick
// (a block is one brick, each of its 4 waves one 1x8x8 slice of 64 voxels).
int mmseg_stem_stats_bricks(int D, int H, int W) { return 4 * (D / SZ) * (H / SY) * (W / SX); }

// mmseg_stem_fwd + InstanceNorm partials of its output (stats [N][mmseg_stem_stats_bricks()][Co][2] = (mean, M2)
// of the stored values over each 64-voxel brick slice; mmseg_instnorm_stats_bricks merges them).
int mmseg_stem_fwd_stats(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N,
                         int D, int H, int W, int Co, float* stats, int dtype, void* stream) {
  MMSEG_REQUIRE(mmseg_stem_ok(cr, Co, D, H, W, ldx, ldy), "stem_fwd: unsupported shape (cr=%d Co=%d %dx%dx%d)", cr,
                Co, D, H, W);
  MMSEG_REQUIRE(Co != 48 || !stats, "stem_fwd: fused statistics need Co = 16 / 32 (power-of-two lane merges)");
  StemArgs g{x, ldx, cr, w, bias, y, ldy, nullptr, 0, nullptr, nullptr, N, D, H, W, Co, stem_kp(cr), 1};
  g.stats = stats;
  const dim3 grid(N * (D / SZ) * (H / SY) * (W / SX));
  hipStream_t s = (hipStream_t)stream;
  mmseg::note_kernel("stem_fwd_kernel");
  auto run = [&](auto tag, auto rn) {
    using T = decltype(tag);
    constexpr int RN = decltype(rn)::value;
    switch (cr) {
      case 1: MMSEG_LAUNCH((stem_fwd_kernel<T, RN, 1>), grid, dim3(256), 0, s, g); break;
      case 2: MMSEG_LAUNCH((stem_fwd_kernel<T, RN, 2>), grid, dim3(256), 0, s, g); break;
      case 3: MMSEG_LAUNCH((stem_fwd_kernel<T, RN, 3>), grid, dim3(256), 0, s, g); break;
      default: MMSEG_LAUNCH((stem_fwd_kernel<T, RN, 4>), grid, dim3(256), 0, s, g); break;
    }
  };
  if (dtype == MMSEG_BF16) {
    if (Co == 16) run(bf16_t{}, std::integral_constant<int, 1>{});
    else if (Co == 48) run(bf16_t{}, std::integral_constant<int, 3>{});
    else run(bf16_t{}, std::integral_constant<int, 2>{});
  } else {
    if (Co == 16) run(float{}, std::integral_constant<int, 1>{});
    else if (Co == 48) run(float{}, std::integral_constant<int, 3>{});
    else run(float{}, std::integral_constant<int, 2>{});
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

int mmseg_stem_wgrad_inb(const void* dy, int lddy, const void* x, int ldx, int cr, const void* inx, int ldinx,
                         const float* inmean, const float* inrstd, const float* incoef, float* part, float* bias_part,
                         int N, int D, int H, int W, int Co, int ksplit, int dtype, void* stream);
int mmseg_stem_fwd_stats(const void* x, int ldx, int cr, const float* w, const float* bias, void* y, int ldy, int N,
                         int D, int H, int W, int Co, float* stats, int dtype, void* stream);

// part[ks][Co][KP] (+ bias_part[ks][Co]); reduce with mmseg_wgrad_reduce(Ca=Co, Ncols=KP, cpad=cr, creal=cr, ntap=27)
int mmseg_stem_wgrad(const void* dy, int lddy, const void* x, int ldx, int cr, float* part, float* bias_part, int N,
                     int D, int H, int W, int Co, int ksplit, int dtype, void* stream) {
  return mmseg_stem_wgrad_inb(dy, lddy, x, ldx, cr, nullptr, 0, nullptr, nullptr, nullptr, part, bias_part, N, D, H,
                              W, Co, ksplit, dtype, stream);
}

// mmseg_stem_wgrad whose dy is the gradient of an InstanceNorm + ReLU OUTPUT (pre-norm input inx, pitch ldinx,
// statistics inmean / inrstd [N][Co], finalised coefficients incoef [N][Co][2] from mmseg_instnorm_bwd_coef): the
// norm's backward is applied while staging dy (in_bwd_apply's values, bit for bit), so its input gradient -- read
// by nothing but this weight gradient -- is never written.  inx null: plain mmseg_stem_wgrad.
int mmseg_stem_wgrad_inb(const void* dy, int lddy, const void* x, int ldx, int cr, const void* inx, int ldinx,
                         const float* inmean, const float* inrstd, const float* incoef, float* part, float* bias_part,
                         int N, int D, int H, int W, int Co, int ksplit, int dtype, void* stream) {
  MMSEG_REQUIRE(mmseg_stem_ok(cr, Co, D, H, W, ldx, lddy), "stem_wgrad: unsupported shape");
  MMSEG_REQUIRE(Co != 48 || (!bias_part && !inx), "stem_wgrad: Co = 48 without bias / fused norm backward only");
  MMSEG_REQUIRE(!inx || (inmean && inrstd && incoef && ldinx % 8 == 0),
                "stem_wgrad_inb: the norm's statistics and coefficients are required, ldinx a multiple of 8");
  StemArgs g{x, ldx, cr, nullptr, nullptr, nullptr, 0, dy, lddy, part, bias_part, N, D, H, W, Co, stem_kp(cr),
             ksplit, inx, ldinx, inmean, inrstd, incoef};
  hipStream_t s = (hipStream_t)stream;
  mmseg::note_kernel("stem_wgrad_kernel");
  const dim3 grid(ksplit), blk(256);
  auto run = [&](auto tag, auto rm) {
    using T = decltype(tag);
    constexpr int RM = decltype(rm)::value;
    if (inx) {
      switch (cr) {
        case 1: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 2, 1, true>), grid, blk, 0, s, g); break;
        case 2: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 4, 2, true>), grid, blk, 0, s, g); break;
        case 3: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 6, 3, true>), grid, blk, 0, s, g); break;
        default: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 8, 4, true>), grid, blk, 0, s, g); break;
      }
      return;
    }
    switch (cr) {
      case 1: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 2, 1>), grid, blk, 0, s, g); break;
      case 2: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 4, 2>), grid, blk, 0, s, g); break;
      case 3: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 6, 3>), grid, blk, 0, s, g); break;
      default: MMSEG_LAUNCH((stem_wgrad_kernel<T, RM, 8, 4>), grid, blk, 0, s, g); break;
    }
  };
  if (dtype == MMSEG_BF16) {
    if (Co == 16) run(bf16_t{}, std::integral_constant<int, 1>{});
    else if (Co == 48) run(bf16_t{}, std::integral_constant<int, 3>{});
    else run(bf16_t{}, std::integral_constant<int, 2>{});
  } else {
    if (Co == 16) run(float{}, std::integral_constant<int, 1>{});
    else if (Co == 48) run(float{}, std::integral_constant<int, 3>{});
    else run(float{}, std::integral_constant<int, 2>{});
  }
  return mmseg::check_launch("stem_wgrad");
}

}  // extern "C"
