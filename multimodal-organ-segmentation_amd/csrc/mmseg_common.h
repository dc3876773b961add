// Common device/host helpers for the MI355X (gfx950) segmentation kernels.
//
// Activation layout inside the engine is NDHWC ("voxel-major, channels
// contiguous"): element (n, v, c) of a tensor with C channels lives at
// base[(n*V + v) * ld + c], where V = D*H*W and ld >= C is the voxel stride.
// ld > C lets a tensor live inside a wider buffer (the decoder's
// [upsampled | skip] concat buffer), so torch.cat never materialises.
//
// Storage type T is float (parity mode) or __bf16 (throughput mode); every
// accumulation is fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <stddef.h>
// the C ABI's declarations: every extern "C" definition in these sources is checked against its prototype
#include "../../include/mmseg_hip.h"

typedef __bf16 bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

enum MmsegDtype { MMSEG_F32 = 0, MMSEG_BF16 = 1 };

#define MMSEG_WAVE 64

// ---------------------------------------------------------------- errors
namespace mmseg {
void set_error(const char* fmt, ...);
int check_launch(const char* what);
// Record the main kernel an entry point launched (mmseg_last_kernel(); the
// per-kernel timer names its regions with it, matching rocprofv3's names).
void note_kernel(const char* name);
// Launch timing (mmseg_timing_begin / _end / _count / _get): while it is on, every kernel goes through
// hipExtLaunchKernelGGL with a start / stop event pair that the runtime stamps from the dispatch itself --
// the kernel's own begin / end, as rocprofv3's kernel trace reports them -- instead of event-record packets
// around the launch, which add the barrier / dispatch latency between them to every kernel.
bool timing_on();
void timing_events(const char* name, hipEvent_t* start, hipEvent_t* stop);
}  // namespace mmseg

// Every kernel launch of the library: hipLaunchKernelGGL, or the timed form while launch timing is on.
#define MMSEG_LAUNCH(K, GRID, BLOCK, SHM, STRM, ...)                                         \
  do {                                                                                     \
    if (mmseg::timing_on()) {                                                              \
      hipEvent_t mmseg_ts_, mmseg_te_;                                                     \
      mmseg::timing_events(#K, &mmseg_ts_, &mmseg_te_);                                    \
      hipExtLaunchKernelGGL(K, GRID, BLOCK, SHM, STRM, mmseg_ts_, mmseg_te_, 0, ##__VA_ARGS__); \
    } else {                                                                               \
      hipLaunchKernelGGL(K, GRID, BLOCK, SHM, STRM, ##__VA_ARGS__);                        \
    }                                                                                      \
  } while (0)

#define MMSEG_REQUIRE(cond, ...)              \
  do {                                        \
    if (!(cond)) {                            \
      mmseg::set_error(__VA_ARGS__);          \
      return 1;                               \
    }                                         \
  } while (0)

// --------------------------------------------------------- 8-wide vectors
// A "v8" is 8 consecutive channels of one voxel: 16 B for bf16, 32 B for f32.
template <typename T> struct V8;
template <> struct V8<float> {
  float v[8];
  __device__ __forceinline__ void load(const float* p) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
  __device__ __forceinline__ void store(float* p) const {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
  __device__ __forceinline__ float get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = x; }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
  }
};
template <> struct V8<bf16_t> {
  bf16x8 v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const bf16x8*>(p); }
  __device__ __forceinline__ void store(bf16_t* p) const { *reinterpret_cast<bf16x8*>(p) = v; }
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = (bf16_t)x; }
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (bf16_t)0.f;
  }
};

template <typename T> __device__ __forceinline__ float to_f(T x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x) { return (T)x; }

// ------------------------------------------------------------ reductions
__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}
__device__ __forceinline__ double wave_sum_d(double x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  return x;
}

static inline int ceil_div(long long a, long long b) { return (int)((a + b - 1) / b); }

// 3x3x3 tap t in [0,27): (kz, ky, kx) = (t/9, (t/3)%3, t%3), offsets -1..1.
__device__ __forceinline__ void tap_delta(int t, int& dz, int& dy, int& dx) {
  dz = t / 9 - 1;
  dy = (t / 3) % 3 - 1;
  dx = t % 3 - 1;
}

// Bitmask of the 27 taps whose neighbour of voxel (z,y,x) is inside the volume.
__device__ __forceinline__ uint32_t tap_valid_mask(int z, int y, int x, int D, int H, int W) {
  uint32_t mz = (z > 0 ? 1u : 0u) | 2u | (z < D - 1 ? 4u : 0u);
  uint32_t my = (y > 0 ? 1u : 0u) | 2u | (y < H - 1 ? 4u : 0u);
  uint32_t mx = (x > 0 ? 1u : 0u) | 2u | (x < W - 1 ? 4u : 0u);
  uint32_t m = 0;
#pragma unroll
  for (int t = 0; t < 27; ++t) {
    int kz = t / 9, ky = (t / 3) % 3, kx = t % 3;
    if (((mz >> kz) & 1u) && ((my >> ky) & 1u) && ((mx >> kx) & 1u)) m |= (1u << t);
  }
  return m;
}

// ---- LDS-DMA (buffer_load ... lds), shared by the conv weight-gradient / brick8 kernels and the window attention
constexpr uint32_t WD_OOB = 0x80000000u;   // buffer offset past every tensor: the DMA writes zeros
typedef int wd_rsrc_t __attribute__((ext_vector_type(4)));
// raw buffer descriptor (base, stride 0, num_records bytes) in SGPRs
__device__ __forceinline__ wd_rsrc_t wd_rsrc(const void* p, uint32_t bytes) {
  const unsigned long long a = (unsigned long long)p;
  wd_rsrc_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32) & 0xffff);
  r[2] = __builtin_amdgcn_readfirstlane((int)bytes);
  r[3] = 0x00020000;
  return r;
}
// one wave-instruction of 16-B LDS-DMA: lane l's chunk lands at LDS byte lds + 16 l.  Issued through inline asm
// so the compiler's waitcnt tracking does not see it: it would otherwise wait for every pending LDS-DMA before
// any LDS read (it cannot tell the stage buffers apart), which serialises the prefetch.  The kernel waits for
// these loads itself (s_waitcnt vmcnt).
__device__ __forceinline__ void wd_dma16(uint32_t lds, uint32_t voff, wd_rsrc_t r) {
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(lds), "v"(voff), "s"(r)
               : "memory", "m0");
}

// XCD-aware block remap (MI355X: 8 XCDs, blocks dealt round-robin b -> b % 8).
// Returns a logical tile id such that each XCD walks a CONTIGUOUS range of
// logical tiles (neighbouring tiles share operand panels in that XCD's L2).
// Bijective for any T (speed only; correctness never depends on placement).
__device__ __forceinline__ int xcd_swizzle(int b, int T) {
  const int xcd = b & 7, j = b >> 3, q = T >> 3, r = T & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + j;
}

// nn.GELU() (exact erf) and its derivative, shared by the elementwise kernels (swin.hip) and the token GEMMs'
// fused epilogues (conv_gemm.hip) so both give the same bits.
__device__ __forceinline__ float mmseg_gelu(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float mmseg_gelu_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * __expf(-0.5f * x * x);
}

// ------------------------------------------------------------ AdamW
// Hyper-parameters of one step, either by value (eager launches) or read from device memory (a captured step
// graph replays the same launch every step; the host refreshes the 8 floats before each replay):
// [decay, omb1, beta2, omb2, eps, step_size, bc2_sqrt, unused].  `skip` (nullable): a device float, the
// step's count of out-of-range labels (summed over the ranks under DP); non-zero leaves p, m, v untouched,
// so a batch the trainer is about to raise on never updates the model.  Shared by the AdamW kernels
// (loss_head.hip) and the fused AdamW + weight pack (conv_gemm.hip): one per-element formula, one set of bits.
struct AdamHyper {
  float decay, omb1, beta2, omb2, eps, step_size, bc2_sqrt, pad;
};
__device__ __forceinline__ bool adamw_load(const AdamHyper& hv, const AdamHyper* hp, const float* skip,
                                           AdamHyper& h) {
  if (skip && *skip != 0.f) return false;
  h = hp ? *hp : hv;
  return true;
}
// torch.optim.AdamW's single-tensor op order (param.mul_(1 - lr wd); exp_avg.lerp_; exp_avg_sq.mul_.addcmul_;
// param.addcdiv_(exp_avg, denom, -step_size)), no contraction
__device__ __forceinline__ float adamw_one(float& pv, float gv, float& mv, float& vv, const AdamHyper& h) {
#pragma clang fp contract(off)
  pv = pv * h.decay;
  mv = h.omb1 < 0.5f ? mv + h.omb1 * (gv - mv) : gv - (gv - mv) * (1.f - h.omb1);
  vv = vv * h.beta2 + (h.omb2 * gv) * gv;
  const float denom = sqrtf(vv) / h.bc2_sqrt + h.eps;
  pv = pv + (-h.step_size) * (mv / denom);
  return pv;
}
// host: one step's hyper-parameters as torch.optim.AdamW (single-tensor, foreach=False) derives them -- the bias
// corrections in double, as Python floats
static inline AdamHyper adamw_hyper(float lr, float beta1, float beta2, float eps, float wd, int step) {
  const double bc1 = 1.0 - pow((double)beta1, step);
  const double bc2 = 1.0 - pow((double)beta2, step);
  AdamHyper h;
  h.decay = (float)(1.0 - (double)lr * (double)wd);
  h.omb1 = (float)(1.0 - (double)beta1);
  h.beta2 = beta2;
  h.omb2 = (float)(1.0 - (double)beta2);
  h.eps = eps;
  h.step_size = (float)(lr / bc1);
  h.bc2_sqrt = (float)sqrt(bc2);
  h.pad = 0.f;
  return h;
}
