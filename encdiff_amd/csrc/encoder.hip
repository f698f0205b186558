// encoder.hip -- concept-encoder kernels (Encoder4 in HIP).
//
// Encoder4.warp (openaimodel_enc.py:1015-1041): latent_unit independent MLPs
//   u_i (B scalars) -> Linear(1,64) -> ELU -> Linear(64,128) -> ELU -> Linear(128,16)
// whose outputs are concatenated to (B, latent_unit*16).  The reference runs them as
// 100 forward / ~300 backward tiny launches; here one workgroup per unit runs the whole
// MLP in fp32 (VALU FMA, weights and WR-row activation chunks in LDS).  The grid is
// (unit, batch chunk): every workgroup runs one unit's MLP on WR rows, so B = 128 fills
// 320 workgroups instead of 20 serial loops.  The backward writes d u and each chunk's
// weight-gradient partials to a caller-provided scratch; a second launch adds the chunks
// in a fixed order into the fp32 gradient arena (deterministic, no atomics).
#include "common.h"

namespace {

constexpr int WT = 256;   // threads
constexpr int WR = 8;     // batch rows per chunk (one workgroup each): 320 workgroups at B = 128
constexpr int H1 = 64, H2 = 128;

ED_DEV float elu_f(float z) { return z > 0.f ? z : expm1f(z); }
ED_DEV float elu_d(float out) { return out > 0.f ? 1.f : out + 1.f; }  // torch elu_backward(is_result)

struct WarpSmem {
  float w1[H1], b1[H1], b2[H2];
  float w2[H2][H1 + 1];        // +1: conflict-free column walks
  float w3[16][H2 + 1];
  float b3[16];
  float h1[WR][H1 + 1];
  float h2[WR][H2 + 1];
  float u[WR];
};

// parameter block of unit i: [W1 64][b1 64][W2 128x64][b2 128][W3 D x 128][b3 D]
ED_DEV void load_unit(WarpSmem& s, const float* P, int D) {
  const float* W1 = P;
  const float* B1 = W1 + H1;
  const float* W2 = B1 + H1;
  const float* B2 = W2 + H2 * H1;
  const float* W3 = B2 + H2;
  const float* B3 = W3 + D * H2;
  for (int i = threadIdx.x; i < H1; i += WT) { s.w1[i] = W1[i]; s.b1[i] = B1[i]; }
  for (int i = threadIdx.x; i < H2; i += WT) s.b2[i] = B2[i];
  for (int i = threadIdx.x; i < H2 * H1; i += WT) s.w2[i / H1][i % H1] = W2[i];
  for (int i = threadIdx.x; i < D * H2; i += WT) s.w3[i / H2][i % H2] = W3[i];
  for (int i = threadIdx.x; i < D; i += WT) s.b3[i] = B3[i];
}

// rows [r0, r0 + nr) of unit `unit`: h1, h2 (post-ELU) into LDS
ED_DEV void warp_hidden(WarpSmem& s, const float* u, long ldu, int unit, int r0, int nr) {
  for (int i = threadIdx.x; i < WR; i += WT) s.u[i] = i < nr ? u[(long)(r0 + i) * ldu + unit] : 0.f;
  __syncthreads();
  for (int e = threadIdx.x; e < WR * H1; e += WT) {
    const int r = e / H1, j = e % H1;
    s.h1[r][j] = elu_f(s.u[r] * s.w1[j] + s.b1[j]);
  }
  __syncthreads();
  for (int e = threadIdx.x; e < WR * H2; e += WT) {
    const int r = e / H2, k = e % H2;
    float a = s.b2[k];
#pragma unroll 8
    for (int j = 0; j < H1; ++j) a += s.h1[r][j] * s.w2[k][j];
    s.h2[r][k] = elu_f(a);
  }
  __syncthreads();
}

__global__ __launch_bounds__(WT) void warp_fwd_kernel(const float* __restrict__ u, long ldu, int batch,
                                                      const float* __restrict__ params, long unit_stride, int D,
                                                      float* __restrict__ out, long ldo) {
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  WarpSmem& s = *reinterpret_cast<WarpSmem*>(smem_raw);
  const int unit = blockIdx.x;
  load_unit(s, params + unit * unit_stride, D);
  {
    const int r0 = blockIdx.y * WR;
    const int nr = min(WR, batch - r0);
    warp_hidden(s, u, ldu, unit, r0, nr);
    for (int e = threadIdx.x; e < nr * D; e += WT) {
      const int r = e / D, m = e % D;
      float a = s.b3[m];
#pragma unroll 8
      for (int k = 0; k < H2; ++k) a += s.h2[r][k] * s.w3[m][k];
      out[(long)(r0 + r) * ldo + unit * D + m] = a;
    }
    __syncthreads();
  }
}

struct WarpBwdSmem {
  WarpSmem f;
  float dout[WR][17];
  float dz2[WR][H2 + 1];
  float dz1[WR][H1 + 1];
};

__global__ __launch_bounds__(WT) void warp_bwd_kernel(const float* __restrict__ u, long ldu, int batch,
                                                      const float* __restrict__ params, long unit_stride, int D,
                                                      const float* __restrict__ dout, long lddo,
                                                      float* __restrict__ du, long lddu,
                                                      float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float smem_raw[];
  WarpBwdSmem& s = *reinterpret_cast<WarpBwdSmem*>(smem_raw);
  const int unit = blockIdx.x, tid = threadIdx.x;
  load_unit(s.f, params + unit * unit_stride, D);
  // register-resident weight-gradient accumulators (fixed ownership -> deterministic)
  float gW2[H2 * H1 / WT];   // 32: entries tid + WT*q of W2 (row-major [k][j])
  float gW3[16 * H2 / WT];   // 8 : entries tid + WT*q of W3 ([m][k], D <= 16)
  float gb2 = 0.f, gW1 = 0.f, gb1 = 0.f, gb3 = 0.f;
#pragma unroll
  for (int q = 0; q < H2 * H1 / WT; ++q) gW2[q] = 0.f;
#pragma unroll
  for (int q = 0; q < 16 * H2 / WT; ++q) gW3[q] = 0.f;
  {
    const int r0 = blockIdx.y * WR;
    const int nr = min(WR, batch - r0);
    warp_hidden(s.f, u, ldu, unit, r0, nr);
    for (int e = tid; e < WR * D; e += WT) {
      const int r = e / D, m = e % D;
      s.dout[r][m] = r < nr ? dout[(long)(r0 + r) * lddo + unit * D + m] : 0.f;
    }
    __syncthreads();
    // dW3[m][k] += sum_r dout[r][m] h2[r][k]; db3
#pragma unroll
    for (int q = 0; q < 16 * H2 / WT; ++q) {
      const int e = tid + WT * q, m = e / H2, k = e % H2;
      if (m < D) {
        float a = 0.f;
        for (int r = 0; r < nr; ++r) a += s.dout[r][m] * s.f.h2[r][k];
        gW3[q] += a;
      }
    }
    if (tid < D) {
      float a = 0.f;
      for (int r = 0; r < nr; ++r) a += s.dout[r][tid];
      gb3 += a;
    }
    // dz2[r][k] = (sum_m dout[r][m] W3[m][k]) * elu'(h2)
    for (int e = tid; e < WR * H2; e += WT) {
      const int r = e / H2, k = e % H2;
      float a = 0.f;
      for (int m = 0; m < D; ++m) a += s.dout[r][m] * s.f.w3[m][k];
      s.dz2[r][k] = r < nr ? a * elu_d(s.f.h2[r][k]) : 0.f;
    }
    __syncthreads();
    // dW2[k][j] += sum_r dz2[r][k] h1[r][j]; db2
#pragma unroll
    for (int q = 0; q < H2 * H1 / WT; ++q) {
      const int e = tid + WT * q, k = e / H1, j = e % H1;
      float a = 0.f;
      for (int r = 0; r < nr; ++r) a += s.dz2[r][k] * s.f.h1[r][j];
      gW2[q] += a;
    }
    if (tid < H2) {
      float a = 0.f;
      for (int r = 0; r < nr; ++r) a += s.dz2[r][tid];
      gb2 += a;
    }
    // dz1[r][j] = (sum_k dz2[r][k] W2[k][j]) * elu'(h1)
    for (int e = tid; e < WR * H1; e += WT) {
      const int r = e / H1, j = e % H1;
      float a = 0.f;
#pragma unroll 8
      for (int k = 0; k < H2; ++k) a += s.dz2[r][k] * s.f.w2[k][j];
      s.dz1[r][j] = r < nr ? a * elu_d(s.f.h1[r][j]) : 0.f;
    }
    __syncthreads();
    // dW1[j] += sum_r dz1[r][j] u[r]; db1[j] += sum_r dz1[r][j]
    if (tid < H1) {
      float a = 0.f, c = 0.f;
      for (int r = 0; r < nr; ++r) { a += s.dz1[r][tid] * s.f.u[r]; c += s.dz1[r][tid]; }
      gW1 += a;
      gb1 += c;
    }
    // du[r] = sum_j dz1[r][j] W1[j]
    if (tid < nr) {
      float a = 0.f;
      for (int j = 0; j < H1; ++j) a += s.dz1[tid][j] * s.f.w1[j];
      du[(long)(r0 + tid) * lddu + unit] = a;
    }
    __syncthreads();
  }
  // this chunk's partial gradients: part[(unit * chunks + chunk) * unit_stride + param]
  float* G = part + ((long)unit * gridDim.y + blockIdx.y) * unit_stride;
  float* gW1p = G;
  float* gb1p = gW1p + H1;
  float* gW2p = gb1p + H1;
  float* gb2p = gW2p + H2 * H1;
  float* gW3p = gb2p + H2;
  float* gb3p = gW3p + D * H2;
  if (tid < H1) { gW1p[tid] = gW1; gb1p[tid] = gb1; }
  if (tid < H2) gb2p[tid] = gb2;
  if (tid < D) gb3p[tid] = gb3;
#pragma unroll
  for (int q = 0; q < H2 * H1 / WT; ++q) gW2p[tid + WT * q] = gW2[q];
#pragma unroll
  for (int q = 0; q < 16 * H2 / WT; ++q) {
    const int e = tid + WT * q;
    if (e < D * H2) gW3p[e] = gW3[q];
  }
}

// grads[unit * stride + i] += sum over chunks (in order) of part[(unit * chunks + c) * stride + i]
__global__ __launch_bounds__(WT) void warp_grad_reduce_kernel(const float* __restrict__ part, int units, int chunks,
                                                             long stride, long n_per_unit, float* __restrict__ grads) {
  const int total = units * (int)n_per_unit;  // < 2^31 (launcher check): 32-bit division
  for (int e = blockIdx.x * WT + threadIdx.x; e < total; e += gridDim.x * WT) {
    const long unit = e / (int)n_per_unit, i = e - unit * n_per_unit;
    float a = 0.f;
    for (int c = 0; c < chunks; ++c) a += part[(unit * chunks + c) * stride + i];
    grads[unit * stride + i] += a;
  }
}

}  // namespace

extern "C" int encdiff_encoder_warp_fwd(const float* u, long ldu, int batch, int units, const float* params,
                                        long unit_stride, int context_dim, float* out, long ldo, void* stream) {
  if (!u || !params || !out || batch <= 0 || units <= 0) return ENCDIFF_ERR_ARG;
  if (context_dim <= 0 || context_dim > 16) return ENCDIFF_ERR_UNSUPPORTED;
  if (unit_stride < 2 * H1 + H2 * H1 + H2 + context_dim * H2 + context_dim) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr = hipFuncSetAttribute((const void*)warp_fwd_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  hipLaunchKernelGGL(warp_fwd_kernel, dim3(units, (batch + WR - 1) / WR), dim3(WT), sizeof(WarpSmem),
                     (hipStream_t)stream, u, ldu, batch, params, unit_stride, context_dim, out, ldo);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_encoder_warp_partials_floats(int batch, int units, long unit_stride) {
  return (int)((long)units * ((batch + WR - 1) / WR) * unit_stride);
}

extern "C" int encdiff_encoder_warp_bwd(const float* u, long ldu, int batch, int units, const float* params,
                                        long unit_stride, int context_dim, const float* dout, long lddo, float* du,
                                        long lddu, float* grads, float* partials, void* stream) {
  if (!u || !params || !dout || !du || !grads || !partials || batch <= 0 || units <= 0) return ENCDIFF_ERR_ARG;
  if (context_dim <= 0 || context_dim > 16) return ENCDIFF_ERR_UNSUPPORTED;
  if (unit_stride < 2 * H1 + H2 * H1 + H2 + context_dim * H2 + context_dim) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr = hipFuncSetAttribute((const void*)warp_bwd_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  const int chunks = (batch + WR - 1) / WR;
  hipLaunchKernelGGL(warp_bwd_kernel, dim3(units, chunks), dim3(WT), sizeof(WarpBwdSmem), (hipStream_t)stream, u,
                     ldu, batch, params, unit_stride, context_dim, dout, lddo, du, lddu, partials);
  ED_CHECK_LAUNCH();
  const long n_per_unit = 2 * H1 + H2 * H1 + H2 + (long)context_dim * H2 + context_dim;
  if ((long)units * n_per_unit >= (1L << 31)) return ENCDIFF_ERR_SHAPE;
  long g = ((long)units * n_per_unit + WT - 1) / WT;
  hipLaunchKernelGGL(warp_grad_reduce_kernel, dim3((unsigned)(g > 1024 ? 1024 : g)), dim3(WT), 0, (hipStream_t)stream,
                     partials, units, chunks, unit_stride, n_per_unit, grads);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

// ------------------------------------------------------------------ trunk head: View + Linear
// Encoder4.encoder[-2:] (openaimodel_enc.py:1012-1013): View((-1, d*16)) of the NCHW trunk
// output then Linear(d*16, latent_unit), on the trunk's NHWC fp32 rows directly: input element
// (image b, channel c, pixel p) sits at r[(b*16 + p)*ldr + c] and is column k = c*16 + p of the
// reference weight W[units][d*16].  fp32 throughout (the reference's precision).
namespace {

constexpr int HPIX = 16;  // the 4x4 grid the trunk ends on

// forward: grid (image, unit quad); wave w of a workgroup owns unit j = 4 * blockIdx.y + w, lane l
// sums columns k = l, l + 64, ... with 8 loads in flight (W rows read coalesced; the image's 8 KB
// of rows stay in L1/L2), then one wave sum.
__global__ __launch_bounds__(256) void head_fwd_kernel(const float* r, long ldr, int d, const float* W,
                                                       const float* bias, int units, float* u, long ldu) {
  const int b = blockIdx.x, K = d * HPIX, lane = threadIdx.x & 63;
  const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (j >= units) return;
  const float* x = r + (long)b * HPIX * ldr;
  const float* w = W + (long)j * K;
  float a = 0.f;
#pragma unroll 8
  for (int e = lane; e < K; e += 64) {  // channel-fastest: the lanes read x rows coalesced
    const int p = e / d, c = e - p * d;
    a += x[(long)p * ldr + c] * w[c * HPIX + p];
  }
  a = wave_sum(a);
  if (lane == 0) u[(long)b * ldu + j] = a + bias[j];
}

// backward, one launch: blocks [0, batch) write dr (bf16 NHWC, the trunk's output gradient) of one
// image each (thread per column k, the image's du in LDS); the next blocks own 16 channels of one
// pixel each, 16 image groups per channel (256 threads): dW[j][k] += sum_b du[b][j] x[b][k], the
// groups added in order through LDS (deterministic, no atomics); the last block adds db.
constexpr int HEAD_CB = 256;
constexpr int HEAD_CW = 16;  // channels per weight-gradient workgroup (x 16 image groups)
#ifndef HEADBWD_SKIP
#define HEADBWD_SKIP 0  // timing builds only (tools/head_bwd_bench.py): 1 no dr blocks, 2 no dW blocks, 4 no db
#endif  // images of du staged in LDS at a time by the dW blocks

template <int UM>
__global__ __launch_bounds__(256) void head_bwd_kernel(const float* r, long ldr, int d, const float* W, int units,
                                                       int batch, const float* du, long lddu, bf16_t* dr, long lddr,
                                                       float* dW, float* db) {
  extern __shared__ float sdu[];  // [batch][UM] (dW blocks; then [4][UM][64] partials) or [UM]
  const int K = d * HPIX;
  // loads are never predicated (a runtime-conditional load is branched around and waited for one
  // at a time): du is zero-padded to UM units in LDS, W rows beyond `units` clamp to row 0
  if ((int)blockIdx.x < batch) {
    if (HEADBWD_SKIP & 1) return;
    const int b = blockIdx.x;
    for (int j = threadIdx.x; j < UM; j += 256) sdu[j] = j < units ? du[(long)b * lddu + j] : 0.f;
    __syncthreads();
#pragma unroll 4
    for (int k = threadIdx.x; k < K; k += 256) {  // (4 outputs' W loads in flight per thread)
      const int c = k / HPIX, p = k - c * HPIX;
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < UM; ++j) a += sdu[j] * W[(long)(j < units ? j : 0) * K + k];
      dr[((long)b * HPIX + p) * lddr + c] = f2bf(a);
    }
    return;
  }
  // a dW block: 64 channels c of one pixel p (k = c * HPIX + p), lanes channel-fastest so the rows
  // of r are read coalesced (256 B per wave per image instead of one 64-B line per lane)
  const int blk = blockIdx.x - batch;
  if (blk == (int)gridDim.x - batch - 1) {
    if (HEADBWD_SKIP & 4) return;
    // the last workgroup: db = sum over images of du, 4 image groups per unit summed in parallel
    // (16 loads in flight per thread) and the group sums added in group order -- a fixed order
    const int j = threadIdx.x & 63, gi = threadIdx.x >> 6, per = (batch + 3) / 4;
    const int i0 = gi * per, i1 = min(batch, i0 + per);
    float a = 0.f;
    if (j < units) {
#pragma unroll 16
      for (int b = i0; b < i1; ++b) a += du[(long)b * lddu + j];
    }
    sdu[gi * 64 + j] = a;
    __syncthreads();
    if (threadIdx.x < units) {
      float t = sdu[threadIdx.x];
#pragma unroll
      for (int k = 1; k < 4; ++k) t += sdu[k * 64 + threadIdx.x];
      db[threadIdx.x] += t;
    }
    return;
  }
  if (HEADBWD_SKIP & 2) return;
  // 16 channels x 16 image groups per workgroup (4 x the workgroups of 64-channel blocks, a quarter
  // of the per-thread image chain); the group partials are added in group order -- a fixed order
  constexpr int CW = HEAD_CW, NG = 256 / CW;
  const int kl = threadIdx.x % CW, q = threadIdx.x / CW;
  const int pp = blk % HPIX, cc = (blk / HPIX) * CW + kl;
  const bool kv = cc < d;
  const int k = cc * HPIX + pp;
  const int qb = (batch + NG - 1) / NG, b0 = q * qb, b1 = min(batch, b0 + qb);
  float acc[UM];  // UM >= units, compile-time indices only (registers)
#pragma unroll
  for (int j = 0; j < UM; ++j) acc[j] = 0.f;
  // du staged HEAD_CB images at a time (any batch fits the LDS); each group still adds its images
  // in increasing order, so the chunking does not change a bit of the result
  for (int c0 = 0; c0 < batch; c0 += HEAD_CB) {
    const int c1 = min(batch, c0 + HEAD_CB);
    __syncthreads();  // the previous chunk is consumed
#pragma unroll 8
    for (int e = threadIdx.x; e < (c1 - c0) * UM; e += 256) {  // (loads in flight, not one per round trip)
      const int b = e / UM, jj = e - b * UM;
      sdu[e] = jj < units ? du[(long)(c0 + b) * lddu + jj] : 0.f;
    }
    __syncthreads();
    if (kv) {
      const int bs = max(b0, c0), be = min(b1, c1);
#pragma unroll 8
      for (int b = bs; b < be; ++b) {
        const float xv = r[((long)b * HPIX + pp) * ldr + cc];
#pragma unroll
        for (int jj = 0; jj < UM; ++jj) acc[jj] += sdu[(b - c0) * UM + jj] * xv;
      }
    }
  }
  __syncthreads();  // sdu is reused for the partials
  float* part = sdu;  // [NG][UM][CW]
#pragma unroll
  for (int jj = 0; jj < UM; ++jj) part[(q * UM + jj) * CW + kl] = acc[jj];
  __syncthreads();
  for (int e = threadIdx.x; e < units * CW; e += 256) {
    const int jj = e / CW, kc = e - jj * CW, c2 = (blk / HPIX) * CW + kc;
    if (c2 >= d) continue;
    float t = part[jj * CW + kc];
#pragma unroll
    for (int g = 1; g < NG; ++g) t += part[(g * UM + jj) * CW + kc];
    dW[(long)jj * K + c2 * HPIX + pp] += t;
  }
}

}  // namespace

extern "C" int encdiff_encoder_head_fwd(const float* r, long ldr, int batch, int d, const float* W, const float* bias,
                                        int units, float* u, long ldu, void* stream) {
  if (!r || !W || !bias || !u || batch <= 0 || d <= 0 || units <= 0 || ldr < d || ldu < units) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(head_fwd_kernel, dim3(batch, (units + 3) / 4), dim3(256), 0, (hipStream_t)stream, r, ldr, d, W, bias,
                     units, u, ldu);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_encoder_head_bwd(const float* r, long ldr, int batch, int d, const float* W, int units,
                                        const float* du, long lddu, void* dr, long lddr, float* dW, float* db,
                                        void* stream) {
  if (!r || !W || !du || !dr || !dW || !db || batch <= 0 || d <= 0 || units <= 0 || units > 64 || lddr < d)
    return ENCDIFF_ERR_ARG;
  const int um = units <= 20 ? 20 : (units <= 40 ? 40 : 64);
  size_t lds = (size_t)(batch < HEAD_CB ? batch : HEAD_CB) * um * sizeof(float);
  if (lds < (size_t)4 * um * 64 * sizeof(float)) lds = (size_t)4 * um * 64 * sizeof(float);  // <= 64 KB
  const int kb = HPIX * ((d + HEAD_CW - 1) / HEAD_CW);  // dW blocks: (channel chunk, pixel)
  auto kern = units <= 20 ? head_bwd_kernel<20> : (units <= 40 ? head_bwd_kernel<40> : head_bwd_kernel<64>);
  hipLaunchKernelGGL(kern, dim3(batch + kb + 1), dim3(256), lds, (hipStream_t)stream, r, ldr, d, W, units, batch, du, lddu,
                     (bf16_t*)dr, lddr, dW, db);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}
