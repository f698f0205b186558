// elementwise.hip -- memory-bound kernels of the EncDiff step: activations,
// GEGLU, resampling, the UNet's 3-channel input/output convolutions, the
// diffusion-side math (timestep embedding, q_sample, L1 loss, DDIM update) and
// the fused AdamW + EMA + bf16 weight pack over the flat parameter arena.
#include "common.h"

namespace {


// One thread per 8 contiguous output elements of a row ([rows][cols], cols % 8 == 0).
__global__ __launch_bounds__(256) void ew_kernel(const EncdiffEwArgs p) {
  const int vpr = p.cols >> 3;
  const int total = p.rows * vpr;  // < 2^31 (launcher check): 32-bit division
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    const int r = idx / vpr;
    const int c = (idx - r * vpr) * 8;
    const bf16_t* X = (const bf16_t*)p.x;
    bf16_t* Y = (bf16_t*)p.y;
    float out[8];
    switch (p.op) {
      case ENCDIFF_EW_COPY: unpack8(*(const uint4*)(X + (long)r * p.ldx + c), out); break;
      case ENCDIFF_EW_SILU: {
        unpack8(*(const uint4*)(X + (long)r * p.ldx + c), out);
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] = silu_f(out[i]);
      } break;
      case ENCDIFF_EW_SILU_BWD: {  // x = pre-activation, x2 = dy
        float d[8];
        unpack8(*(const uint4*)(X + (long)r * p.ldx + c), out);
        unpack8(*(const uint4*)((const bf16_t*)p.x2 + (long)r * p.ldx2 + c), d);
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] = d[i] * silu_grad(out[i]);
      } break;
      case ENCDIFF_EW_GEGLU: {  // x: [rows][2*cols]
        float a[8], g[8];
        unpack8(*(const uint4*)(X + (long)r * p.ldx + c), a);
        unpack8(*(const uint4*)(X + (long)r * p.ldx + p.cols + c), g);
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] = a[i] * gelu_erf(g[i]);
      } break;
      case ENCDIFF_EW_GEGLU_BWD: {  // x: [rows][2*cols] proj output, x2 = dy [rows][cols]; y: [rows][2*cols]
        float a[8], g[8], d[8], da[8], dg[8];
        unpack8(*(const uint4*)(X + (long)r * p.ldx + c), a);
        unpack8(*(const uint4*)(X + (long)r * p.ldx + p.cols + c), g);
        unpack8(*(const uint4*)((const bf16_t*)p.x2 + (long)r * p.ldx2 + c), d);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          da[i] = d[i] * gelu_erf(g[i]);
          dg[i] = d[i] * a[i] * gelu_erf_grad(g[i]);
        }
        *(uint4*)(Y + (long)r * p.ldy + c) = pack8(da);
        *(uint4*)(Y + (long)r * p.ldy + p.cols + c) = pack8(dg);
        continue;
      }
      case ENCDIFF_EW_ADD: {
        float d[8];
        unpack8(*(const uint4*)(X + (long)r * p.ldx + c), out);
        unpack8(*(const uint4*)((const bf16_t*)p.x2 + (long)r * p.ldx2 + c), d);
#pragma unroll
        for (int i = 0; i < 8; ++i) out[i] += d[i];
      } break;
      case ENCDIFF_EW_RESAMPLE: {  // output pixel r at (h, w)
        const int hw = p.h * p.w;
        const int b = r / hw, rem = r - b * hw, y = rem / p.w, x = rem - (rem / p.w) * p.w;
        if (p.resample == ENCDIFF_RESAMPLE_DOWN2) {
          const int W2 = 2 * p.w;
          const long r0 = ((long)b * 2 * p.h + 2 * y) * W2 + 2 * x;
          float t[8];
          unpack8(*(const uint4*)(X + r0 * p.ldx + c), out);
          unpack8(*(const uint4*)(X + (r0 + 1) * p.ldx + c), t);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] += t[i];
          unpack8(*(const uint4*)(X + (r0 + W2) * p.ldx + c), t);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] += t[i];
          unpack8(*(const uint4*)(X + (r0 + W2 + 1) * p.ldx + c), t);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] = (out[i] + t[i]) * 0.25f;
        } else {
          const long rs = ((long)b * (p.h >> 1) + (y >> 1)) * (p.w >> 1) + (x >> 1);
          unpack8(*(const uint4*)(X + rs * p.ldx + c), out);
        }
      } break;
      case ENCDIFF_EW_RESAMPLE_BWD: {  // adjoint: output (h, w) = forward source dims
        const int hw = p.h * p.w;
        const int b = r / hw, rem = r - b * hw, y = rem / p.w, x = rem - (rem / p.w) * p.w;
        if (p.resample == ENCDIFF_RESAMPLE_DOWN2) {  // fwd (h,w)->(h/2,w/2): dx = 0.25 dy[y/2][x/2]
          const long rs = ((long)b * (p.h >> 1) + (y >> 1)) * (p.w >> 1) + (x >> 1);
          unpack8(*(const uint4*)(X + rs * p.ldx + c), out);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] *= 0.25f;
        } else {  // fwd (h,w)->(2h,2w) nearest: dx = sum of the 4 children
          const int W2 = 2 * p.w;
          const long r0 = ((long)b * 2 * p.h + 2 * y) * W2 + 2 * x;
          float t[8];
          unpack8(*(const uint4*)(X + r0 * p.ldx + c), out);
          unpack8(*(const uint4*)(X + (r0 + 1) * p.ldx + c), t);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] += t[i];
          unpack8(*(const uint4*)(X + (r0 + W2) * p.ldx + c), t);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] += t[i];
          unpack8(*(const uint4*)(X + (r0 + W2 + 1) * p.ldx + c), t);
#pragma unroll
          for (int i = 0; i < 8; ++i) out[i] += t[i];
        }
      } break;
      case ENCDIFF_EW_F32_TO_BF16: {
        const float* Xf = (const float*)p.x + (long)r * p.ldx + c;
        const float4 a = *(const float4*)Xf, b = *(const float4*)(Xf + 4);
        out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
        out[4] = b.x; out[5] = b.y; out[6] = b.z; out[7] = b.w;
      } break;
      case ENCDIFF_EW_BF16_TO_F32: {
        unpack8(*(const uint4*)(X + (long)r * p.ldx + c), out);
        float* Yf = (float*)p.y + (long)r * p.ldy + c;
        if (p.accumulate) {
#pragma unroll
          for (int i = 0; i < 8; ++i) Yf[i] += out[i];
        } else {
          *(float4*)Yf = make_float4(out[0], out[1], out[2], out[3]);
          *(float4*)(Yf + 4) = make_float4(out[4], out[5], out[6], out[7]);
        }
        continue;
      }
      default: return;
    }
    bf16_t* yp = Y + (long)r * p.ldy + c;
    if (p.accumulate) {
      float prev[8];
      unpack8(*(const uint4*)yp, prev);
#pragma unroll
      for (int i = 0; i < 8; ++i) out[i] += prev[i];
    }
    *(uint4*)yp = pack8(out);
  }
}

// ------------------------------------------------ 3-channel convolutions (VALU)
// input conv (cin = 3): x fp32 NCHW -> y bf16 NHWC.  thread per (pixel, co)
// input conv (cin <= 4, fp32 NCHW) -> bf16 NHWC: thread per output pixel, the cin*9 input
// taps in registers, all cout outputs accumulated 8 at a time and written as 16-byte vectors.
__global__ __launch_bounds__(256) void small_conv_in_fwd(const EncdiffSmallConvArgs p) {
  __shared__ float w[64 * 36 + 64];
  const int CO = p.cout, CI = p.cin, HW = p.h * p.w, KW = CI * 9;
  for (int i = threadIdx.x; i < CO * KW; i += 256) w[i] = p.weight[i];
  for (int i = threadIdx.x; i < CO; i += 256) w[CO * KW + i] = p.bias[i];
  __syncthreads();
  const long total = (long)p.batch * HW;
  for (long pix = blockIdx.x * 256L + threadIdx.x; pix < total; pix += (long)gridDim.x * 256) {
    const int b = (int)(pix / HW), rem = (int)(pix - (long)b * HW);
    const int y = rem / p.w, x = rem - y * p.w;
    const float* X = (const float*)p.x + (long)b * CI * HW;
    float in[36];
#pragma unroll
    for (int ci = 0; ci < 4; ++ci)
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        in[ci * 9 + t] = (ci < CI && yy >= 0 && yy < p.h && xx >= 0 && xx < p.w) ? X[(long)ci * HW + yy * p.w + xx] : 0.f;
      }
    bf16_t* Y = (bf16_t*)p.y + pix * p.ldy;
    for (int c0 = 0; c0 < CO; c0 += 8) {
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float* wr = w + (c0 + j) * KW;
        float a = w[CO * KW + c0 + j];
#pragma unroll
        for (int k = 0; k < 36; ++k)
          if (k < KW) a += wr[k] * in[k];
        acc[j] = a;
      }
      *(uint4*)(Y + c0) = pack8(acc);
    }
  }
}

// output conv (cout = 3): x bf16 NHWC [pix][cin] -> y fp32 NCHW.  thread per pixel
__global__ __launch_bounds__(256) void small_conv_out_fwd(const EncdiffSmallConvArgs p) {
  __shared__ float w[3 * 9 * 512 + 3];
  const int CO = p.cout, CI = p.cin, HW = p.h * p.w;
  // weight reordered to [co][tap][ci]
  for (int i = threadIdx.x; i < CO * CI * 9; i += 256) {
    const int co = i / (CI * 9), rem = i - co * CI * 9, ci = rem / 9, t = rem - ci * 9;
    w[(co * 9 + t) * CI + ci] = p.weight[i];
  }
  for (int i = threadIdx.x; i < CO; i += 256) w[CO * CI * 9 + i] = p.bias[i];
  __syncthreads();
  const long total = (long)p.batch * HW;
  for (long pix = blockIdx.x * 256L + threadIdx.x; pix < total; pix += (long)gridDim.x * 256) {
    const int b = (int)(pix / HW), rem = (int)(pix - (long)b * HW);
    const int y = rem / p.w, x = rem - y * p.w;
    float acc[3] = {0.f, 0.f, 0.f};
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (yy < 0 || yy >= p.h || xx < 0 || xx >= p.w) continue;
      const bf16_t* src = (const bf16_t*)p.x + ((long)b * HW + yy * p.w + xx) * p.ldx;
      for (int ci = 0; ci < CI; ci += 8) {
        float v[8];
        unpack8(*(const uint4*)(src + ci), v);
#pragma unroll
        for (int co = 0; co < 3; ++co)
#pragma unroll
          for (int i = 0; i < 8; ++i) acc[co] += v[i] * w[(co * 9 + t) * CI + ci + i];
      }
    }
    float* Y = (float*)p.y + (long)b * CO * HW + rem;
    for (int co = 0; co < CO; ++co) Y[(long)co * HW] = acc[co] + w[CO * CI * 9 + co];
  }
}

// output conv (cout = 3), many-lane form: thread per (pixel, 8-channel chunk); the 2^vshift
// chunk lanes of a pixel are adjacent in the wave and fold their 3 partial sums with xor
// shuffles.  8-16x the threads of the thread-per-pixel kernel (which filled half the CUs at
// 32K pixels and ran its 9 x CI/8 vector loads serially).
__global__ __launch_bounds__(256) void small_conv_out_fwd_lanes(const EncdiffSmallConvArgs p, int vshift) {
  extern __shared__ __attribute__((aligned(16))) float w[];  // [3][9][CI] + 3 biases (sized at launch)
  const int CO = p.cout, CI = p.cin, HW = p.h * p.w;
  // staged in destination order (consecutive lanes -> consecutive LDS words, no conflicts)
  for (int j = threadIdx.x; j < CO * CI * 9; j += 256) {
    const int ct = j / CI, ci = j - ct * CI, co = ct / 9, t = ct - co * 9;
    w[j] = p.weight[(co * CI + ci) * 9 + t];
  }
  for (int i = threadIdx.x; i < CO; i += 256) w[CO * CI * 9 + i] = p.bias[i];
  __syncthreads();
  const int V = 1 << vshift;
  // 32-bit indices (the launcher checks batch * HW * V < 2^31): no 64-bit divisions
  const int total = p.batch * HW * V;  // a multiple of V: lane groups are all-or-none valid
  for (int base = blockIdx.x * 256; base < total; base += gridDim.x * 256) {
    const int idx = base + threadIdx.x;
    const bool valid = idx < total;
    const int pix = idx >> vshift;
    const int ci0 = (idx & (V - 1)) * 8;
    const int b = pix / HW, rem = pix - b * HW;
    const int y = rem / p.w, x = rem - y * p.w;
    float acc[3] = {0.f, 0.f, 0.f};
    if (valid) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
        if (yy < 0 || yy >= p.h || xx < 0 || xx >= p.w) continue;
        float v[8];
        unpack8(*(const uint4*)((const bf16_t*)p.x + ((long)b * HW + yy * p.w + xx) * p.ldx + ci0), v);
#pragma unroll
        for (int co = 0; co < 3; ++co) {
          // (co * 9 + t) * CI + ci0 is a multiple of 8 floats: two 16-byte LDS reads
          const float4* wr = (const float4*)(w + (co * 9 + t) * CI + ci0);
          const float4 w0 = wr[0], w1 = wr[1];
          acc[co] += v[0] * w0.x + v[1] * w0.y + v[2] * w0.z + v[3] * w0.w + v[4] * w1.x + v[5] * w1.y +
                     v[6] * w1.z + v[7] * w1.w;
        }
      }
    }
    for (int o = V >> 1; o > 0; o >>= 1)
#pragma unroll
      for (int co = 0; co < 3; ++co) acc[co] += __shfl_xor(acc[co], o, 64);
    if (valid && ci0 == 0) {
      float* Y = (float*)p.y + (long)b * CO * HW + rem;
      for (int co = 0; co < CO; ++co) Y[(long)co * HW] = acc[co] + w[CO * CI * 9 + co];
    }
  }
}

// dx of the output conv: dy fp32 NCHW [b][3][hw] -> dx bf16 NHWC [pix][cin].  thread per (pix, 8 ci)
__global__ __launch_bounds__(256) void small_conv_out_dgrad(const EncdiffSmallConvArgs p) {
  extern __shared__ __attribute__((aligned(16))) float w[];  // [3][9][CI], sized at launch
  const int CO = p.cout, CI = p.cin, HW = p.h * p.w;
  // [co][tap][ci]: the chunk lanes of a pixel read consecutive 32-byte runs (the source
  // [co][ci][tap] order put them 72 floats apart: bank conflicts)
  for (int j = threadIdx.x; j < CO * CI * 9; j += 256) {  // destination order: conflict-free
    const int ct = j / CI, ci = j - ct * CI, co = ct / 9, t = ct - co * 9;
    w[j] = p.weight[(co * CI + ci) * 9 + t];
  }
  __syncthreads();
  const int vpp = CI / 8;
  const int total = p.batch * HW * vpp;  // < 2^31 (launcher check): 32-bit index math
  for (int idx = blockIdx.x * 256 + threadIdx.x; idx < total; idx += gridDim.x * 256) {
    const int pix = idx / vpp;
    const int ci0 = (idx - pix * vpp) * 8;
    const int b = pix / HW, rem = pix - b * HW;
    const int y = rem / p.w, x = rem - y * p.w;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const float* DY = (const float*)p.dy + (long)b * CO * HW;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      // output pixel o = in - (t offset): y_out = y - (t/3 - 1)
      const int yo = y - (t / 3 - 1), xo = x - (t % 3 - 1);
      if (yo < 0 || yo >= p.h || xo < 0 || xo >= p.w) continue;
#pragma unroll
      for (int co = 0; co < 3; ++co) {
        if (co >= CO) break;
        const float d = DY[co * HW + yo * p.w + xo];
        const float4* wr = (const float4*)(w + (co * 9 + t) * CI + ci0);  // 32-byte aligned
        const float4 w0 = wr[0], w1 = wr[1];
        acc[0] += d * w0.x; acc[1] += d * w0.y; acc[2] += d * w0.z; acc[3] += d * w0.w;
        acc[4] += d * w1.x; acc[5] += d * w1.y; acc[6] += d * w1.z; acc[7] += d * w1.w;
      }
    }
    *(uint4*)((bf16_t*)p.dx + pix * p.lddx + ci0) = pack8(acc);
  }
}

// weight/bias gradient of either small conv.  One block per group of images; each
// grid (ceil(NW/256), ceil(batch/ipb)): a thread owns ONE output weight o = (co, ci, tap)
// and sums over the pixels of the block's images; partial sums are atomically added.
// in-conv: x fp32 NCHW, dy bf16 NHWC [pix][co];  out-conv: x bf16 NHWC, dy fp32 NCHW.
__global__ __launch_bounds__(256) void small_conv_wgrad(const EncdiffSmallConvArgs p, int imgs_per_block) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int CO = p.cout, CI = p.cin, H = p.h, W = p.w, HW = H * W;
  float* xs = sm;              // [CI][HW]
  float* ds = sm + CI * HW;    // [CO][HW]
  const int NW = CO * CI * 9;
  const int o = blockIdx.x * 256 + threadIdx.x;
  const bool live = o < NW;
  const int co = live ? o / (CI * 9) : 0, rem = o - co * CI * 9, ci = rem / 9, t = rem - ci * 9;
  const int oy = t / 3 - 1, ox = t % 3 - 1;
  const int y0 = max(0, -oy), y1 = min(H, H - oy), x0 = max(0, -ox), x1 = min(W, W - ox);
  const bool do_bias = blockIdx.x == 0 && threadIdx.x < CO && p.dbias;
  float acc = 0.f, bacc = 0.f;
  const int b0 = blockIdx.y * imgs_per_block;
  for (int b = b0; b < min(p.batch, b0 + imgs_per_block); ++b) {
    __syncthreads();
    for (int i = threadIdx.x; i < CI * HW; i += 256) {
      const int c = i / HW, px = i - c * HW;
      xs[i] = p.x_f32 ? ((const float*)p.x)[(long)b * CI * HW + i]
                      : bf2f(((const bf16_t*)p.x)[((long)b * HW + px) * p.ldx + c]);
    }
    for (int i = threadIdx.x; i < CO * HW; i += 256) {
      const int c = i / HW, px = i - c * HW;
      ds[i] = p.dy_f32 ? ((const float*)p.dy)[(long)b * CO * HW + i]
                       : bf2f(((const bf16_t*)p.dy)[((long)b * HW + px) * p.lddy + c]);
    }
    __syncthreads();
    if (live) {
      const float* dr = ds + co * HW;
      const float* xr = xs + ci * HW + oy * W + ox;
      for (int y = y0; y < y1; ++y)
        for (int x = x0; x < x1; ++x) acc += dr[y * W + x] * xr[y * W + x];
    }
    if (do_bias) {
      const float* dr = ds + threadIdx.x * HW;
      for (int px = 0; px < HW; ++px) bacc += dr[px];
    }
  }
  if (live) atomicAdd(p.dweight + o, acc);
  if (do_bias) atomicAdd(p.dbias + threadIdx.x, bacc);
}

// ------------------------------------------------ diffusion math
__global__ void temb_kernel(const long long* t, int batch, int dim, float max_period, bf16_t* out) {
  const int half = dim / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch * half) return;
  const int b = i / half, k = i - b * half;
  // util.py:185-189, fp32: exp(-ln(max_period) * k / half)
  const float freq = __expf((-logf(max_period) * (float)k) / (float)half);
  const float arg = (float)t[b] * freq;
  out[b * dim + k] = f2bf(cosf(arg));
  out[b * dim + half + k] = f2bf(sinf(arg));
}

__global__ void qsample_kernel(const float* x0, const float* eps, const long long* t, const float* sa,
                               const float* s1a, int batch, int per, float* xt, const float* x0_scale) {
  const long n = (long)batch * per;
  const float sc = x0_scale ? *x0_scale : 1.f;  // get_first_stage_encoding's scale_factor, folded in
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int b = (int)(i / per);
    const long long tt = t[b];
    xt[i] = sa[tt] * (sc * x0[i]) + s1a[tt] * eps[i];
  }
}

// L1 loss: block b writes loss_simple[b] to partials; the LAST block to arrive (device-scope
// ticket after write-through partial stores, acquire in the last block, as in bn.hip) folds the batch in a fixed order and resets the
// ticket.  No memset and no float atomics: graph-replay safe and bitwise reproducible.
__global__ __launch_bounds__(256) void l1_kernel(const float* pred, const float* eps, const long long* t,
                                                 const float* lvlb, int batch, int per, float lsw, float* out2,
                                                 float* grad, float* partials, unsigned int* counter) {
  __shared__ float red[8];
  __shared__ int last;
  const int b = blockIdx.x;
  float s = 0.f;
  const float gscale = lsw / ((float)batch * per);
  for (int i = threadIdx.x; i < per; i += 256) {
    const long j = (long)b * per + i;
    const float d = pred[j] - eps[j];
    s += fabsf(d);
    if (grad) grad[j] = (d > 0.f ? gscale : (d < 0.f ? -gscale : 0.f));
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    // loss_simple[b], stored write-through (sc1): visible to the last arriver (which acquires)
    // without an agent release writing back the L2 (the gradient seed just written by every wave)
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)partials, 0, 0x7FFFFFF0, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, (red[0] + red[1] + red[2] + red[3]) / (float)per),
                                          rs, b * 4, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned tk = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = tk == (unsigned)batch - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  if (!last) return;
  float a = 0.f, v = 0.f;  // thread i: samples i, i + 256, ... in order
  for (int k = threadIdx.x; k < batch; k += 256) {
    const float ls = partials[k];
    a += ls;
    v += lvlb[t[k]] * ls;
  }
  a = wave_sum(a);
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) { red[threadIdx.x >> 6] = a; red[4 + (threadIdx.x >> 6)] = v; }
  __syncthreads();
  if (threadIdx.x == 0) {
    out2[0] = lsw * (((red[0] + red[1]) + red[2]) + red[3]) / (float)batch;
    out2[1] = (((red[4] + red[5]) + red[6]) + red[7]) / (float)batch;
    *counter = 0u;
  }
}

__global__ void ddim_kernel(const float* x, const float* e, const float* z, int n, float a_t, float a_prev,
                            float sigma, float s1, float* xp, float* px0) {
  const float rs = 1.f / sqrtf(a_t);
  const float sap = sqrtf(a_prev);
  const float dcoef = sqrtf(1.f - a_prev - sigma * sigma);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float ee = e[i];
    const float p0 = (x[i] - s1 * ee) * rs;
    if (px0) px0[i] = p0;
    xp[i] = sap * p0 + dcoef * ee + (z ? sigma * z[i] : 0.f);
  }
}

__global__ void ddim_indexed_kernel(const float* x, const float* e, const float* z, int n, const float* coef,
                                    const int* index, float* xp, float* px0) {
  const int idx = *index;
  const float a_t = coef[4 * idx], a_prev = coef[4 * idx + 1], sigma = coef[4 * idx + 2], s1 = coef[4 * idx + 3];
  const float rs = 1.f / sqrtf(a_t);
  const float sap = sqrtf(a_prev);
  const float dcoef = sqrtf(1.f - a_prev - sigma * sigma);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float ee = e[i];
    const float p0 = (x[i] - s1 * ee) * rs;
    if (px0) px0[i] = p0;
    xp[i] = sap * p0 + dcoef * ee + (z ? sigma * z[i] : 0.f);
  }
}

__global__ void index_dec_kernel(int* index) { *index -= 1; }

// ------------------------------------------------ input path
// Block per image: the uint8 HWC image is staged through LDS with 16-byte loads, then
// written as fp32 CHW with float4 stores.
__global__ __launch_bounds__(256) void gather_u8_kernel(const uint8_t* __restrict__ pool, long long n_images,
                                                        int hw, int c, const long long* __restrict__ perm,
                                                        const long long* step, int steps_per_epoch,
                                                        float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t img[];
  const int b = blockIdx.x, B = gridDim.x;
  const long long s = step ? *step : 0;
  const long long id = perm[(s % steps_per_epoch) * B + b];
  const int nbytes = hw * c;
  const uint8_t* src = pool + (id < 0 ? 0 : (id >= n_images ? n_images - 1 : id)) * (long long)nbytes;
  if ((nbytes & 15) == 0 && (((uintptr_t)src) & 15) == 0) {
    for (int i = threadIdx.x; i < nbytes / 16; i += 256) ((uint4*)img)[i] = ((const uint4*)src)[i];
  } else {
    for (int i = threadIdx.x; i < nbytes; i += 256) img[i] = src[i];
  }
  __syncthreads();
  float* o = out + (long long)b * nbytes;
  const int n4 = nbytes >> 2;  // hw % 4 == 0 checked on the host
  for (int i = threadIdx.x; i < n4; i += 256) {
    const int e = i * 4, ch = e / hw, px = e - ch * hw;
    float4 v;
    v.x = ((float)img[(px + 0) * c + ch] / 255.f - 0.5f) / 0.5f;
    v.y = ((float)img[(px + 1) * c + ch] / 255.f - 0.5f) / 0.5f;
    v.z = ((float)img[(px + 2) * c + ch] / 255.f - 0.5f) / 0.5f;
    v.w = ((float)img[(px + 3) * c + ch] / 255.f - 0.5f) / 0.5f;
    ((float4*)o)[i] = v;
  }
}

__global__ void counter_inc_kernel(long long* counter) { *counter += 1; }

// ------------------------------------------------ step prologue (RNG + zeroing + counters)
// Philox4x32-10 (Salmon et al., SC'11): 4 x 32-bit counter, 2 x 32-bit key, 10 rounds.
ED_DEV uint4 philox10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t h0 = __umulhi(0xD2511F53u, c.x), l0 = 0xD2511F53u * c.x;
    const uint32_t h1 = __umulhi(0xCD9E8D57u, c.z), l1 = 0xCD9E8D57u * c.z;
    c = make_uint4(h1 ^ c.y ^ k0, l1, h0 ^ c.w ^ k1, l0);
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}
ED_DEV float u01(uint32_t x) { return ((float)x + 1.0f) * 2.3283064365386963e-10f; }  // (0, 1]

__global__ __launch_bounds__(256) void step_prologue_kernel(const EncdiffStepPrologueArgs a) {
  const long long ctr = *a.rng_counter;
  const uint32_t k0 = (uint32_t)a.seed, k1 = (uint32_t)(a.seed >> 32);
  const uint32_t c_lo = (uint32_t)ctr, c_hi = (uint32_t)((unsigned long long)ctr >> 32);
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x, gs = (long long)gridDim.x * blockDim.x;
  if (a.noise) {
    for (long long q = gid; q * 4 < a.n_noise; q += gs) {
      const uint4 r = philox10(make_uint4((uint32_t)q, c_lo, c_hi, 0u), k0, k1);
      const float m0 = sqrtf(-2.f * logf(u01(r.x))), m1 = sqrtf(-2.f * logf(u01(r.z)));
      float s0, c0, s1, c1;
      sincospif(2.f * u01(r.y), &s0, &c0);
      sincospif(2.f * u01(r.w), &s1, &c1);
      const float v[4] = {m0 * c0, m0 * s0, m1 * c1, m1 * s1};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (q * 4 + j < a.n_noise) a.noise[q * 4 + j] = v[j];
    }
  }
  if (a.t) {
    for (long long b = gid; b < a.batch; b += gs) {
      const uint4 r = philox10(make_uint4((uint32_t)b, c_lo, c_hi, 1u), k0, k1);
      a.t[b] = (long long)(((unsigned long long)r.x * (unsigned)a.timesteps) >> 32);
    }
  }
  for (int j = 0; j < a.njobs; ++j) {
    const EncdiffZeroJob z = a.jobs[j];
    const long long per = z.row_bytes >> 4, n = z.rows * per;
    if (z.ld_bytes == z.row_bytes || z.rows == 1) {  // contiguous: a flat 16-B sweep (the gradient arena)
      uint4* p = (uint4*)z.ptr;
      for (long long i = gid; i < n; i += gs) p[i] = make_uint4(0u, 0u, 0u, 0u);
    } else {  // strided rows: 32-bit row / column split (the host keeps rows and per < 2^31)
      for (long long i = gid; i < n; i += gs) {
        const uint32_t r = (uint32_t)i / (uint32_t)per, cc = (uint32_t)i - r * (uint32_t)per;
        *(uint4*)((char*)z.ptr + (long long)r * z.ld_bytes + (long long)cc * 16) = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  // the last workgroup advances the counters (every workgroup read *rng_counter before its ticket).
  // Only that read must be complete before the ticket: a wait on this wave's memory operations,
  // not a __threadfence (an agent release writes back the XCD L2's dirty lines -- here the freshly
  // zeroed arena, 2048 times: it was most of the kernel's time).  The counters reach the next
  // kernels at the kernel boundary.
  __syncthreads();
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int tk = atomicAdd(a.done, 1);
    if (tk == (int)gridDim.x - 1) {
      *a.rng_counter = ctr + 1;
      if (a.data_step) *a.data_step += 1;
      *a.done = 0;
    }
  }
}


// ------------------------------------------------ optimizer
__global__ __launch_bounds__(256) void adamw_ema_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                        float* __restrict__ m, float* __restrict__ v,
                                                        float* __restrict__ ema, long long n,
                                                        const float* __restrict__ hyper, long long ema_n,
                                                        bf16_t* __restrict__ mirror) {
  const float lr = hyper[0], b1 = hyper[1], b2 = hyper[2], eps = hyper[3], wd = hyper[4];
  const float step_size = hyper[5], inv_bc2_sqrt = hyper[6], omd = hyper[7];
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n4; i += (long long)gridDim.x * blockDim.x) {
    float4 pp = ((float4*)p)[i], gg = ((const float4*)g)[i], mm = ((float4*)m)[i], vv = ((float4*)v)[i];
    float* pa = &pp.x; const float* ga = &gg.x; float* ma = &mm.x; float* va = &vv.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // torch.optim.AdamW (single-tensor): decoupled decay, lerp for m, addcmul for v
      pa[k] *= (1.f - lr * wd);
      ma[k] = ma[k] + (1.f - b1) * (ga[k] - ma[k]);
      va[k] = b2 * va[k] + (1.f - b2) * ga[k] * ga[k];
      const float denom = sqrtf(va[k]) * inv_bc2_sqrt + eps;
      pa[k] -= step_size * ma[k] / denom;
    }
    ((float4*)p)[i] = pp; ((float4*)m)[i] = mm; ((float4*)v)[i] = vv;
    if (mirror) ((uint2*)mirror)[i] = make_uint2(pack2(pa[0], pa[1]), pack2(pa[2], pa[3]));  // bf16 GEMM copy
    if (ema && 4 * i < ema_n) {  // LitEma.forward (ema.py:37-42): s -= (1 - decay) (s - p)
      float4 ee = ((float4*)ema)[i];
      float* ea = &ee.x;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * i + k < ema_n) ea[k] -= omd * (ea[k] - pa[k]);
      ((float4*)ema)[i] = ee;
    }
  }
}

__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ src, bf16_t* __restrict__ dst,
                                                   const EncdiffPackJob* __restrict__ jobs) {
  const EncdiffPackJob j = jobs[blockIdx.y];
  const int total = j.rows * j.cols;  // < 2^31 (host)
  const int stride = gridDim.x * 256;
  if (j.kind == 0 && (total & 7) == 0 && (j.src_off & 3) == 0 && (j.dst_off & 7) == 0) {
    // plain copy-cast: 8 elements per lane (two float4 loads, one 16-byte store)
    const float* s0 = src + j.src_off;
    bf16_t* d0 = dst + j.dst_off;
    for (int i = (blockIdx.x * 256 + threadIdx.x) * 8; i < total; i += stride * 8) {
      float v[8];
      const float4 a = *(const float4*)(s0 + i), b = *(const float4*)(s0 + i + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
      *(uint4*)(d0 + i) = pack8(v);
    }
    return;
  }
  if (j.kind == 6) {
    // transposed copy-cast (the SpatialTransformer backward kernels' B operands, st_bwd.hip):
    // src [rows][cols] -> dst [cols][rows], 32 x 32 tiles through LDS (coalesced both ways)
    __shared__ float tile[32][33];
    const int tr = (j.rows + 31) / 32, tc = (j.cols + 31) / 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    for (int t = blockIdx.x; t < tr * tc; t += gridDim.x) {
      const int r0 = (t / tc) * 32, c0 = (t % tc) * 32;
      __syncthreads();
      for (int k = ty; k < 32; k += 8) {
        const int r = r0 + k, c = c0 + tx;
        tile[k][tx] = (r < j.rows && c < j.cols) ? src[j.src_off + (long)r * j.cols + c] : 0.f;
      }
      __syncthreads();
      for (int k = ty; k < 32; k += 8) {
        const int c = c0 + k, r = r0 + tx;
        if (c < j.cols && r < j.rows) dst[j.dst_off + (long)c * j.rows + r] = f2bf(tile[tx][k]);
      }
    }
    return;
  }
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += stride) {
    const int r = i / j.cols, c = i - r * j.cols;  // 32-bit: the 64-bit divide was most of the time
    long s;
    if (j.kind == 1) {  // conv [co][ci][3][3] -> [co][tap][ci]; c = tap*cin + ci
      const int tap = c / j.cin, ci = c - tap * j.cin;
      s = (long)r * j.cols + ci * 9 + tap;
    } else if (j.kind == 2) {  // conv [co][cin][taps] -> [co][tap][8], channels cin..7 zero
      const int taps = j.cols >> 3, tap = c >> 3, ci = c & 7;
      if (ci >= j.cin) {
        dst[j.dst_off + i] = 0;
        continue;
      }
      s = (long)r * j.cin * taps + ci * taps + tap;
    } else if (j.kind >= 3) {
      // split-bf16 operands (bf16x3): w = hi + lo, hi = bf16(w), lo = bf16(w - hi).  Per tap the
      // K block is [hi | hi | lo] (kind 3: src [co][tap][cin] row-major, cin channels per block;
      // kind 4: src [co][cin][taps], cin <= 8, blocks of 8 channels zero-padded) or, kind 5
      // (1x1 conv + identity residual), [hi | hi | lo | I | I] over src [co][cin].  Paired with
      // activations stored [hi | lo | hi] (and the residual input as [hi | lo]) one GEMM computes
      // a_hi w_hi + a_lo w_hi + a_hi w_lo (+ x_hi + x_lo): ~16 significant bits per product.
      const int cb = j.kind == 4 ? 8 : j.cin;  // channels per block
      const int tap = c / (j.kind == 5 ? 5 * cb : 3 * cb);
      const int rem = c - tap * (j.kind == 5 ? 5 * cb : 3 * cb);
      const int blk = rem / cb, ci = rem - blk * cb;
      if (blk >= 3) {  // kind 5 identity blocks
        dst[j.dst_off + i] = f2bf(ci == r ? 1.f : 0.f);
        continue;
      }
      if (ci >= j.cin) {  // kind 4 channel padding
        dst[j.dst_off + i] = 0;
        continue;
      }
      const int taps = j.kind == 4 ? j.cols / 24 : (j.kind == 5 ? 1 : j.cols / (3 * j.cin));
      const long si = j.kind == 4 ? (long)r * j.cin * taps + ci * taps + tap : (long)r * taps * j.cin + tap * j.cin + ci;
      const float w = src[j.src_off + si];
      const float hi = bf16_round(w);
      dst[j.dst_off + i] = f2bf(blk < 2 ? hi : w - hi);
      continue;
    } else {
      s = i;
    }
    dst[j.dst_off + i] = f2bf(src[j.src_off + s]);
  }
}

// A workgroup owns 32 columns; its 8 row slices (32 lanes each) sum rows slice, slice + 8, ...
// (4 independent accumulators per lane keep loads in flight), then the slices are added in
// a fixed order through LDS: deterministic, and 8x more workgroups than one thread per column.
__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* part, long ld, int rows, int cols,
                                                              const int* idx, float* grad) {
  __shared__ float red[8][32];
  const int cl = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int j = blockIdx.x * 32 + cl;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (j < cols) {
    int r = sl;
    for (; r + 24 < rows; r += 32) {
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(long)(r + 8 * u) * ld + j];
    }
    for (; r < rows; r += 8) a[0] += part[(long)r * ld + j];
  }
  red[sl][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (sl == 0 && j < cols) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][cl];
    grad[idx[j]] += t;
  }
}

// workgroup cap of the output-conv kernels: each workgroup stages all 3 x 9 x CI weights in
// LDS first, so a few grid-stride rounds per workgroup amortise that (tools/kbench.py sconv)
int sconv_wgs() {
  static const int v = [] {
    const char* e = getenv("ENCDIFF_SCONV_WGS");
    return e ? atoi(e) : 1024;
  }();
  return v;
}

int grid_for(long n, int per_thread = 1) {
  long g = (n / per_thread + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

extern "C" int encdiff_elementwise(const EncdiffEwArgs* a, void* stream) {
  if (!a || !a->x || !a->y) return ENCDIFF_ERR_ARG;
  if (a->dtype == ENCDIFF_DT_F32) return ed_elementwise_f32(a, (hipStream_t)stream);
  if (a->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_ARG;
  if (a->cols % 8 || (long)a->rows * (a->cols / 8) >= (1L << 31)) return ENCDIFF_ERR_SHAPE;
  hipLaunchKernelGGL(ew_kernel, dim3(grid_for((long)a->rows * a->cols, 8)), dim3(256), 0, (hipStream_t)stream, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_small_conv_fwd(const EncdiffSmallConvArgs* a, void* stream) {
  if (!a || !a->x || !a->y || !a->weight || !a->bias) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const long pix = (long)a->batch * a->h * a->w;
  if (a->x_f32 && !a->y_f32) {  // input conv
    if (a->cin > 4 || a->cout > 64 || a->cout % 8 || a->ldy % 8) return ENCDIFF_ERR_SHAPE;
    hipLaunchKernelGGL(small_conv_in_fwd, dim3(grid_for(pix)), dim3(256), 0, s, *a);
  } else if (!a->x_f32 && a->y_f32) {  // output conv
    if (a->cout > 3 || a->cin > 512 || a->cin % 8) return ENCDIFF_ERR_SHAPE;
    const int v = a->cin / 8;
    if ((v & (v - 1)) == 0 && pix * v < (1L << 31)) {  // 32-bit indices in the lane kernel  // power-of-two chunk count (<= 64): lane groups within a wave
      int vshift = 0;
      while ((1 << vshift) < v) ++vshift;
      const size_t lds = (size_t)(3 * 9 * a->cin + 3) * sizeof(float);
      hipLaunchKernelGGL(small_conv_out_fwd_lanes, dim3(std::min(grid_for(pix * v), sconv_wgs())), dim3(256), lds, s,
                         *a, vshift);
    } else {
      hipLaunchKernelGGL(small_conv_out_fwd, dim3(grid_for(pix)), dim3(256), 0, s, *a);
    }
  } else {
    return ENCDIFF_ERR_UNSUPPORTED;
  }
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_small_conv_bwd(const EncdiffSmallConvArgs* a, void* stream) {
  if (!a || !a->x || !a->dy || !a->weight) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int HW = a->h * a->w;
  if (a->dx) {
    if (!a->dy_f32 || a->cout > 3 || a->cin % 8) return ENCDIFF_ERR_UNSUPPORTED;
    if (a->cin > 512) return ENCDIFF_ERR_SHAPE;  // LDS weight copy holds 3 x 9 x 512
    if ((long)a->batch * HW * (a->cin / 8) >= (1L << 31)) return ENCDIFF_ERR_SHAPE;  // 32-bit indices
    hipLaunchKernelGGL(small_conv_out_dgrad, dim3(std::min(grid_for((long)a->batch * HW * (a->cin / 8)), sconv_wgs())),
                       dim3(256), (size_t)3 * 9 * a->cin * sizeof(float), s, *a);
    ED_CHECK_LAUNCH();
  }
  if (a->dweight) {
    const size_t lds = (size_t)(a->cin + a->cout) * HW * sizeof(float);
    if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
    static const hipError_t attr = hipFuncSetAttribute((const void*)small_conv_wgrad,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)attr;
    const int ipb = 2, nw = a->cout * a->cin * 9;
    hipLaunchKernelGGL(small_conv_wgrad, dim3((nw + 255) / 256, (a->batch + ipb - 1) / ipb), dim3(256), lds, s, *a,
                       ipb);
    ED_CHECK_LAUNCH();
  }
  return ENCDIFF_OK;
}

extern "C" int encdiff_timestep_embedding(const long long* t, int batch, int dim, float max_period, void* out,
                                          void* stream) {
  if (!t || !out || dim % 2) return ENCDIFF_ERR_ARG;
  const int n = batch * dim / 2;
  hipLaunchKernelGGL(temb_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, t, batch, dim,
                     max_period, (bf16_t*)out);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_q_sample(const float* x0, const float* eps, const long long* t, const float* sa,
                                const float* s1a, int batch, int per, float* xt, void* stream) {
  if (!x0 || !eps || !t || !sa || !s1a || !xt) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(qsample_kernel, dim3(grid_for((long)batch * per)), dim3(256), 0, (hipStream_t)stream, x0, eps,
                     t, sa, s1a, batch, per, xt, (const float*)nullptr);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_q_sample_scaled(const float* x0, const float* x0_scale, const float* eps, const long long* t,
                                       const float* sa, const float* s1a, int batch, int per, float* xt,
                                       void* stream) {
  if (!x0 || !x0_scale || !eps || !t || !sa || !s1a || !xt) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(qsample_kernel, dim3(grid_for((long)batch * per)), dim3(256), 0, (hipStream_t)stream, x0, eps,
                     t, sa, s1a, batch, per, xt, x0_scale);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_l1_loss(const float* pred, const float* eps, const long long* t, const float* lvlb, int batch,
                               int per, float lsw, float* out2, float* grad, float* partials, unsigned int* counter,
                               void* stream) {
  if (!pred || !eps || !t || !lvlb || !out2 || !partials || !counter || batch <= 0 || per <= 0) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(l1_kernel, dim3(batch), dim3(256), 0, (hipStream_t)stream, pred, eps, t, lvlb, batch, per, lsw,
                     out2, grad, partials, counter);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_ddim_step(const float* x, const float* e, const float* noise, int n, float a_t, float a_prev,
                                 float sigma, float s1, float* xp, float* px0, void* stream) {
  if (!x || !e || !xp) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(ddim_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, e, noise, n, a_t, a_prev,
                     sigma, s1, xp, px0);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_ddim_step_indexed(const float* x, const float* e, const float* noise, int n, const float* coef,
                                         int* index, int advance, float* xp, float* px0, void* stream) {
  if (!x || !e || !xp || !coef || !index) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(ddim_indexed_kernel, dim3(grid_for(n)), dim3(256), 0, s, x, e, noise, n, coef, index, xp, px0);
  ED_CHECK_LAUNCH();
  if (advance) {
    hipLaunchKernelGGL(index_dec_kernel, dim3(1), dim3(1), 0, s, index);
    ED_CHECK_LAUNCH();
  }
  return ENCDIFF_OK;
}

extern "C" int encdiff_gather_images_u8(const void* pool, long long n_images, int h, int w, int c,
                                        const long long* perm, long long* step, int steps_per_epoch, int batch,
                                        int advance, float* out, void* stream) {
  if (!pool || !perm || !out || batch <= 0 || steps_per_epoch <= 0 || n_images <= 0) return ENCDIFF_ERR_ARG;
  if ((h * w) % 4 || (long)h * w * c > 64 * 1024) return ENCDIFF_ERR_SHAPE;
  if (advance && !step) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(gather_u8_kernel, dim3(batch), dim3(256), (size_t)h * w * c, s, (const uint8_t*)pool, n_images,
                     h * w, c, perm, step, steps_per_epoch, out);
  ED_CHECK_LAUNCH();
  if (advance) {
    hipLaunchKernelGGL(counter_inc_kernel, dim3(1), dim3(1), 0, s, step);
    ED_CHECK_LAUNCH();
  }
  return ENCDIFF_OK;
}

extern "C" int encdiff_step_prologue(const EncdiffStepPrologueArgs* a, void* stream) {
  if (!a || !a->rng_counter || !a->done || a->njobs < 0 || (a->njobs && !a->jobs)) return ENCDIFF_ERR_ARG;
  if (a->t && (a->batch <= 0 || a->timesteps <= 0)) return ENCDIFF_ERR_ARG;
  if (a->noise && a->n_noise <= 0) return ENCDIFF_ERR_ARG;
  // workgroups: the zeroing (a 155 MB gradient arena) dominates -- 2048 x 256 threads x 16 B
  hipLaunchKernelGGL(step_prologue_kernel, dim3(a->njobs ? 2048 : 64), dim3(256), 0, (hipStream_t)stream, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_adamw_ema(float* p, const float* g, float* m, float* v, float* ema, long long n,
                                 const float* hyper, long long ema_n, void* stream) {
  return encdiff_adamw_ema_mirror(p, g, m, v, ema, n, hyper, ema_n, nullptr, stream);
}

extern "C" int encdiff_adamw_ema_mirror(float* p, const float* g, float* m, float* v, float* ema, long long n,
                                        const float* hyper, long long ema_n, void* mirror, void* stream) {
  if (!p || !g || !m || !v || !hyper || n % 4 || ((uintptr_t)mirror & 7)) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(adamw_ema_kernel, dim3(grid_for(n, 4)), dim3(256), 0, (hipStream_t)stream, p, g, m, v, ema, n,
                     hyper, ema_n, (bf16_t*)mirror);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_pack_weights(const float* src, void* dst, const EncdiffPackJob* jobs, int njobs, void* stream) {
  if (!src || !dst || !jobs || njobs <= 0 || njobs > 65535) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(pack_kernel, dim3(128, njobs), dim3(256), 0, (hipStream_t)stream, src, (bf16_t*)dst, jobs);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

// conv weight-gradient fold (see encdiff_grad_fold): one thread per arena weight
__global__ __launch_bounds__(256) void grad_fold_kernel(const float* dw, int co, int cin, int cpad, int taps, float* db,
                                                        float* gw, float* gb) {
  const int n = co * cin * taps;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    const int o = i / (cin * taps), r = i - o * cin * taps, c = r / taps, t = r - c * taps;
    gw[i] += dw[((long)o * taps + t) * cpad + c];
  }
  if (db && blockIdx.x == 0 && threadIdx.x < co) {
    gb[threadIdx.x] += db[threadIdx.x];
    db[threadIdx.x] = 0.f;
  }
}

extern "C" int encdiff_grad_fold(const float* dw, int co, int cin, int cpad, int taps, float* db, float* gw, float* gb,
                                 void* stream) {
  if (!dw || !gw || (db && !gb) || co <= 0 || cin <= 0 || cin > cpad || taps <= 0 || co > 256)
    return ENCDIFF_ERR_ARG;
  const int n = co * cin * taps;
  hipLaunchKernelGGL(grad_fold_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, dw, co, cin, cpad,
                     taps, db, gw, gb);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_reduce_partials(const float* part, long ld, int rows, int cols, const int* idx, float* grad,
                                       void* stream) {
  if (!part || !idx || !grad || cols <= 0) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(reduce_partials_kernel, dim3((cols + 31) / 32), dim3(256), 0, (hipStream_t)stream, part, ld,
                     rows, cols, idx, grad);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}
