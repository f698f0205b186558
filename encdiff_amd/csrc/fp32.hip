// fp32.hip -- the reference-precision (fp32) forward of the denoiser, SURVEY §8(b) convention (5).
//
// The reference computes in fp32 (main_val.py:525; TF32 matmuls on its GPUs).  The product path
// runs bf16 activations with fp32 accumulation; these kernels run the SAME entry points with
// fp32 activations (the args' `dtype` = ENCDIFF_DT_F32) so that the denoiser forward can be held
// to the fp32 tolerance (1e-4 rel-L2) against the reference's own output:
//   GEMM / conv   encdiff_gemm                : v_mfma_f32_16x16x4_f32 (exact f32 products,
//                                              fp32 accumulation), 64x64 tiles, implicit im2col
//   GroupNorm     encdiff_groupnorm_fwd       : two-pass statistics, FiLM, SiLU
//   LayerNorm     encdiff_layernorm_fwd       : two-pass statistics
//   attention     encdiff_attention_fwd       : exact softmax (max-subtracted, expf), fp32 P V
//   elementwise   encdiff_elementwise         : SiLU, GEGLU (erf), add, resample, copy
//   plus encdiff_timestep_embedding_f32 and encdiff_nchw_rows_f32 (layout changes).
// Forward only (a parity / reference-precision sampling path; the training step is bf16).
// Replaces the same reference computations as the bf16 entry points (see include/encdiff_hip.h).
#include <math.h>

#include "common.h"

namespace {

constexpr int FBM = 64, FBN = 64, FBK = 16;

struct F32Conv {
  int sh, lh, lw, hs, ws;  // nearest-up shift, conv-input limits, source dims
  uint32_t hw, w, cin;
};

// one output tile of C = alpha * A B (+bias)(+resid), A rows [M][K] (ROWK) or implicit im2col of an
// NHWC fp32 source (IM2COL, 3x3 pad 1, optional nearest x2), B = W [N][K] (ROWK).
template <int AM>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const EncdiffGemmArgs p, const F32Conv cv) {
  __shared__ float As[FBK][FBM + 4];
  __shared__ float Bs[FBK][FBN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * FBM, n0 = blockIdx.y * FBN;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const float* A = (const float*)p.a;
  const float* Bw = (const float*)p.b;
  // staging: thread -> (row, 4 consecutive k)
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const int am = m0 + lr, bn = n0 + lr;
  int ab = 0, ay = 0, ax = 0;
  if (AM == ENCDIFF_OPA_IM2COL && am < p.M) {
    ab = am / (int)cv.hw;
    const int r = am - ab * (int)cv.hw;
    ay = r / (int)cv.w;
    ax = r - ay * (int)cv.w;
  }
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < p.K; k0 += FBK) {
    const int k = k0 + lk;
    float4 av = make_float4(0.f, 0.f, 0.f, 0.f), bv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (am < p.M && k < p.K) {  // K % 4 == 0 (host): the 4 values are in range together
      if (AM == ENCDIFF_OPA_ROWK) {
        av = *(const float4*)(A + (long)am * p.lda + k);
      } else {  // IM2COL: k = tap * cin + c, cin % 4 == 0
        const int tap = k / (int)cv.cin, c = k - tap * (int)cv.cin;
        const int ty = tap / 3, tx = tap - 3 * ty;
        const int ys = ay + ty - 1, xs = ax + tx - 1;
        if ((unsigned)ys < (unsigned)cv.lh && (unsigned)xs < (unsigned)cv.lw) {
          const long row = ((long)ab * cv.hs + (ys >> cv.sh)) * cv.ws + (xs >> cv.sh);
          av = *(const float4*)(A + row * p.conv.ld_src + c);
        }
      }
    }
    if (bn < p.N && k < p.K) bv = *(const float4*)(Bw + (long)bn * p.ldb + k);
    __syncthreads();
    As[lk][lr] = av.x; As[lk + 1][lr] = av.y; As[lk + 2][lr] = av.z; As[lk + 3][lr] = av.w;
    Bs[lk][lr] = bv.x; Bs[lk + 1][lr] = bv.y; Bs[lk + 2][lr] = bv.z; Bs[lk + 3][lr] = bv.w;
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < FBK; kk += 4) {
      // 16x16x4: lane l holds A[l & 15][k = l >> 4] and B[k = l >> 4][l & 15]
      const int ki = kk + (lane >> 4);
      float af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = As[ki][wr + 16 * i + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = Bs[ki][wc + 16 * j + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }
  const float* R = (const float*)p.resid;
  float* Cp = (float*)p.c;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wc + 16 * j + (lane & 15);
      if (col >= p.N) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = m0 + wr + 16 * i + 4 * (lane >> 4) + q;
        if (row >= p.M) continue;
        float v = p.alpha * acc[i][j][q];
        if (p.bias) v += p.bias[col];
        if (R) v += R[(long)row * p.ld_resid + col];
        float* cp = Cp + (long)row * p.ldc + col;
        *cp = p.c_mode == ENCDIFF_OUT_F32_ACCUM ? *cp + v : v;
      }
    }
}

// GroupNorm (+FiLM)(+SiLU), fp32 rows [batch*hw][ld]: one workgroup per (image, group), two-pass
// statistics (mean, then the centred variance), as torch.nn.functional.group_norm in fp32.
__global__ __launch_bounds__(256) void gn_f32_kernel(const EncdiffGroupNormArgs p) {
  __shared__ float red[4];
  const int b = blockIdx.x / p.groups, g = blockIdx.x - b * p.groups;
  const int cpg = p.c / p.groups, n = cpg * p.hw;
  const float* X = (const float*)p.x + (long)b * p.hw * p.ldx + g * cpg;
  auto at = [&](int i) -> float { const int px = i / cpg, c = i - px * cpg; return X[(long)px * p.ldx + c]; };
  auto bsum = [&](float v) -> float {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
  };
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += at(i);
  const float mean = bsum(s) / (float)n;
  float q = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) { const float d = at(i) - mean; q += d * d; }
  const float rstd = 1.f / sqrtf(bsum(q) / (float)n + p.eps);
  if (threadIdx.x == 0) { p.stats[2 * blockIdx.x] = mean; p.stats[2 * blockIdx.x + 1] = rstd; }
  float* Y = (float*)p.y + (long)b * p.hw * p.ldy + g * cpg;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int px = i / cpg, cl = i - px * cpg, c = g * cpg + cl;
    float v = (at(i) - mean) * rstd * p.gamma[c] + p.beta[c];
    if (p.film) v = v * (1.f + p.film[(long)b * p.ld_film + c]) + p.film[(long)b * p.ld_film + p.c + c];
    if (p.silu) v = v / (1.f + expf(-v));
    Y[(long)px * p.ldy + cl] = v;
  }
}

// LayerNorm over the channels of fp32 rows: one wave per row, two-pass statistics.
__global__ __launch_bounds__(256) void ln_f32_kernel(const EncdiffLayerNormArgs p) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= p.rows) return;
  const float* X = (const float*)p.x + (long)row * p.ldx;
  float s = 0.f;
  for (int c = lane; c < p.c; c += 64) s += X[c];
  const float mean = wave_sum(s) / (float)p.c;
  float q = 0.f;
  for (int c = lane; c < p.c; c += 64) { const float d = X[c] - mean; q += d * d; }
  const float rstd = 1.f / sqrtf(wave_sum(q) / (float)p.c + p.eps);
  float* Y = (float*)p.y + (long)row * p.ldy;
  for (int c = lane; c < p.c; c += 64) Y[c] = (X[c] - mean) * rstd * p.gamma[c] + p.beta[c];
  if (p.stats && lane == 0) { p.stats[2L * row] = mean; p.stats[2L * row + 1] = rstd; }
}

// softmax(q k^T * scale) v per (image, head): one thread per query row, keys / values staged in
// LDS in chunks of 128; exact softmax (running max, expf rescale), fp32 throughout.
constexpr int AKC = 128;
template <int DH>
__global__ __launch_bounds__(64) void attn_f32_kernel(const EncdiffAttnArgs p) {
  __shared__ float Ks[AKC][DH + 1];
  __shared__ float Vs[AKC][DH + 1];
  const int bh = blockIdx.y, b = bh / p.heads, h = bh - b * p.heads;
  const int qi = blockIdx.x * 64 + threadIdx.x;
  const bool live = qi < p.sq;
  float q[DH], o[DH];
  const float* Q = (const float*)p.q + ((long)b * p.sq + (live ? qi : 0)) * p.ldq + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) { q[d] = Q[d] * p.scale; o[d] = 0.f; }
  float mx = -INFINITY, den = 0.f;
  const float* Kg = (const float*)p.k + (long)b * p.sk * p.ldk + h * DH;
  const float* Vg = (const float*)p.v + (long)b * p.sk * p.ldv + h * DH;
  for (int k0 = 0; k0 < p.sk; k0 += AKC) {
    const int nk = min(AKC, p.sk - k0);
    __syncthreads();
    for (int i = threadIdx.x; i < nk * DH; i += 64) {
      const int r = i / DH, d = i - r * DH;
      Ks[r][d] = Kg[(long)(k0 + r) * p.ldk + d];
      Vs[r][d] = Vg[(long)(k0 + r) * p.ldv + d];
    }
    __syncthreads();
    for (int j = 0; j < nk; ++j) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s += q[d] * Ks[j][d];
      if (s > mx) {
        const float c = expf(mx - s);
        den *= c;
#pragma unroll
        for (int d = 0; d < DH; ++d) o[d] *= c;
        mx = s;
      }
      const float e = expf(s - mx);
      den += e;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] += e * Vs[j][d];
    }
  }
  if (!live) return;
  float* O = (float*)p.o + ((long)b * p.sq + qi) * p.ldo + h * DH;
  const float inv = 1.f / den;
#pragma unroll
  for (int d = 0; d < DH; ++d) O[d] = o[d] * inv;
  if (p.lse) p.lse[(long)bh * p.sq + qi] = mx + logf(den);
}

// elementwise ops on fp32 [rows][cols] (strided rows)
__global__ __launch_bounds__(256) void ew_f32_kernel(const EncdiffEwArgs p) {
  const long n = (long)p.rows * p.cols;
  const float* X = (const float*)p.x;
  const float* X2 = (const float*)p.x2;
  float* Y = (float*)p.y;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int r = (int)(i / p.cols), c = (int)(i - (long)r * p.cols);
    float v;
    switch (p.op) {
      case ENCDIFF_EW_COPY: v = X[(long)r * p.ldx + c]; break;
      case ENCDIFF_EW_SILU: { const float z = X[(long)r * p.ldx + c]; v = z / (1.f + expf(-z)); break; }
      case ENCDIFF_EW_GEGLU: {  // value half first, gate second (attention.py:42-44)
        const float a = X[(long)r * p.ldx + c], g = X[(long)r * p.ldx + p.cols + c];
        v = a * (0.5f * g * (1.f + erff(g * 0.70710678118654752f)));
        break;
      }
      case ENCDIFF_EW_ADD: v = X[(long)r * p.ldx + c] + X2[(long)r * p.ldx2 + c]; break;
      case ENCDIFF_EW_RESAMPLE: {  // r = output pixel (b, y, x) of (h, w); down: avgpool2, up: nearest
        const int hw = p.h * p.w, b = r / hw, rr = r - b * hw, y = rr / p.w, x = rr - y * p.w;
        if (p.resample == ENCDIFF_RESAMPLE_DOWN2) {
          const int W2 = 2 * p.w;
          const long s0 = ((long)b * 2 * p.h + 2 * y) * W2 + 2 * x;
          v = 0.25f * (X[s0 * p.ldx + c] + X[(s0 + 1) * p.ldx + c] + X[(s0 + W2) * p.ldx + c] +
                       X[(s0 + W2 + 1) * p.ldx + c]);
        } else {
          const long s = ((long)b * (p.h / 2) + y / 2) * (p.w / 2) + x / 2;
          v = X[s * p.ldx + c];
        }
        break;
      }
      default: v = 0.f;
    }
    float* yp = Y + (long)r * p.ldy + c;
    *yp = p.accumulate ? *yp + v : v;
  }
}

__global__ void temb_f32_kernel(const long long* t, int batch, int dim, float max_period, float* out) {
  const int half = dim / 2;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= batch * half) return;
  const int b = i / half, k = i - b * half;
  // util.py:185-189 in fp32: freqs = exp(-ln(max_period) * arange(half) / half); args = t * freqs
  const float freq = expf((-logf(max_period) * (float)k) / (float)half);
  const float arg = (float)t[b] * freq;
  out[b * dim + k] = cosf(arg);
  out[b * dim + half + k] = sinf(arg);
}

// dir 0: NCHW [batch][c][hw] -> rows [batch*hw][ld] (channels c..cpad-1 zero); dir 1: back
__global__ void nchw_rows_f32_kernel(const float* x, int batch, int c, int hw, int cpad, float* y, long ld, int dir) {
  const long n = (long)batch * hw * cpad;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const long px = i / cpad;
    const int ch = (int)(i - px * cpad);
    const long b = px / hw, s = px - b * hw;
    if (dir == 0) {
      y[px * ld + ch] = ch < c ? x[(b * c + ch) * hw + s] : 0.f;
    } else if (ch < c) {
      y[(b * c + ch) * hw + s] = x[px * ld + ch];
    }
  }
}

int grid256(long n) {
  const long g = (n + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

int ed_gemm_f32(const EncdiffGemmArgs* p, hipStream_t s) {
  if (p->M <= 0 || p->N <= 0 || p->K <= 0 || p->K % 4) return ENCDIFF_ERR_SHAPE;
  if (p->b_mode != ENCDIFF_OPB_ROWK || (p->a_mode != ENCDIFF_OPA_ROWK && p->a_mode != ENCDIFF_OPA_IM2COL))
    return ENCDIFF_ERR_UNSUPPORTED;
  if ((p->c_mode != ENCDIFF_OUT_F32 && p->c_mode != ENCDIFF_OUT_F32_ACCUM) || p->split_k > 1 || p->bias_grad ||
      p->gn_stats || p->ln_y)
    return ENCDIFF_ERR_UNSUPPORTED;
  if (p->lda % 4 || p->ldb % 4 || ((uintptr_t)p->a & 15) || ((uintptr_t)p->b & 15)) return ENCDIFF_ERR_SHAPE;
  F32Conv cv{};
  if (p->a_mode == ENCDIFF_OPA_IM2COL) {
    const int rs = p->conv.resample;
    if (rs != ENCDIFF_RESAMPLE_NONE && rs != ENCDIFF_RESAMPLE_UP2) return ENCDIFF_ERR_UNSUPPORTED;
    if (p->conv.cin % 4 || p->conv.ld_src % 4 || p->K != 9 * p->conv.cin ||
        (long)p->M != (long)p->conv.batch * p->conv.h * p->conv.w)
      return ENCDIFF_ERR_SHAPE;
    if (rs == ENCDIFF_RESAMPLE_UP2 && ((p->conv.h | p->conv.w) & 1)) return ENCDIFF_ERR_SHAPE;
    cv.sh = rs == ENCDIFF_RESAMPLE_UP2 ? 1 : 0;
    cv.lh = p->conv.h;
    cv.lw = p->conv.w;
    cv.hs = p->conv.h >> cv.sh;
    cv.ws = p->conv.w >> cv.sh;
    cv.hw = (uint32_t)(p->conv.h * p->conv.w);
    cv.w = (uint32_t)p->conv.w;
    cv.cin = (uint32_t)p->conv.cin;
  }
  dim3 grid((p->M + FBM - 1) / FBM, (p->N + FBN - 1) / FBN);
  if (p->a_mode == ENCDIFF_OPA_ROWK)
    hipLaunchKernelGGL(gemm_f32_kernel<ENCDIFF_OPA_ROWK>, grid, dim3(256), 0, s, *p, cv);
  else
    hipLaunchKernelGGL(gemm_f32_kernel<ENCDIFF_OPA_IM2COL>, grid, dim3(256), 0, s, *p, cv);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_groupnorm_fwd_f32(const EncdiffGroupNormArgs* a, hipStream_t s) {
  if (!a->x || !a->y || !a->stats || !a->gamma || !a->beta) return ENCDIFF_ERR_ARG;
  if (a->groups <= 0 || a->c % a->groups || a->in_stats) return ENCDIFF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(gn_f32_kernel, dim3(a->batch * a->groups), dim3(256), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_layernorm_fwd_f32(const EncdiffLayerNormArgs* a, hipStream_t s) {
  if (!a->x || !a->y || !a->gamma || !a->beta) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(ln_f32_kernel, dim3((a->rows + 3) / 4), dim3(256), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_attention_fwd_f32(const EncdiffAttnArgs* a, hipStream_t s) {
  if (!a->q || !a->k || !a->v || !a->o || a->fp8_qk) return ENCDIFF_ERR_ARG;
  dim3 grid((a->sq + 63) / 64, a->batch * a->heads);
  switch (a->dh) {
    case 8: hipLaunchKernelGGL(attn_f32_kernel<8>, grid, dim3(64), 0, s, *a); break;
    case 16: hipLaunchKernelGGL(attn_f32_kernel<16>, grid, dim3(64), 0, s, *a); break;
    case 32: hipLaunchKernelGGL(attn_f32_kernel<32>, grid, dim3(64), 0, s, *a); break;
    case 64: hipLaunchKernelGGL(attn_f32_kernel<64>, grid, dim3(64), 0, s, *a); break;
    default: return ENCDIFF_ERR_SHAPE;
  }
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_elementwise_f32(const EncdiffEwArgs* a, hipStream_t s) {
  if (a->op != ENCDIFF_EW_COPY && a->op != ENCDIFF_EW_SILU && a->op != ENCDIFF_EW_GEGLU && a->op != ENCDIFF_EW_ADD &&
      a->op != ENCDIFF_EW_RESAMPLE)
    return ENCDIFF_ERR_UNSUPPORTED;
  if (a->op == ENCDIFF_EW_ADD && !a->x2) return ENCDIFF_ERR_ARG;
  if (a->op == ENCDIFF_EW_RESAMPLE && a->resample != ENCDIFF_RESAMPLE_DOWN2 && a->resample != ENCDIFF_RESAMPLE_UP2)
    return ENCDIFF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(ew_f32_kernel, dim3(grid256((long)a->rows * a->cols)), dim3(256), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_timestep_embedding_f32(const long long* t, int batch, int dim, float max_period, float* out,
                                              void* stream) {
  if (!t || !out || dim % 2) return ENCDIFF_ERR_ARG;
  const int n = batch * dim / 2;
  hipLaunchKernelGGL(temb_f32_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, t, batch, dim,
                     max_period, out);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_nchw_rows_f32(const float* x, int batch, int c, int hw, int cpad, float* y, long ld, int dir,
                                     void* stream) {
  if (!x || !y || c > cpad || ld < cpad || (dir != 0 && dir != 1)) return ENCDIFF_ERR_ARG;
  hipLaunchKernelGGL(nchw_rows_f32_kernel, dim3(grid256((long)batch * hw * cpad)), dim3(256), 0, (hipStream_t)stream,
                     x, batch, c, hw, cpad, y, ld, dir);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}
