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

// one output tile of C = alpha * A B (+bias)(+resid) (+= for F32_ACCUM), fp32 operands, exact f32
// MFMA products.  A: ROWK (A[m][k]), ROWM (A stored [k][m]: the k-outer operand of a weight
// gradient) or IM2COL (implicit im2col of an NHWC fp32 source, 3x3 pad 1, optional nearest x2);
// B: ROWK (B stored [n][k], weights), ROWN (B stored [k][n]: an input gradient's weight operand or
// a weight gradient's activations), IM2COL (B[k = pixel][n = (tap, c)] of an NHWC source: the
// 3x3 conv weight gradient) or CONV_DGRAD (B[k = (tap, co)][n = ci] = W[co][(8 - tap) * N + ci]:
// the flipped kernel of the conv input gradient).  bias_grad (ROWM only): += sum_k A[m][k].
struct Im2F32 {
  const float* src;
  long ld;
  F32Conv cv;
  // element (pixel m, column k = tap * cin + c) of the im2col matrix
  ED_DEV float at(int m, int k) const {
    const int b = m / (int)cv.hw, r = m - b * (int)cv.hw, y = r / (int)cv.w, x = r - y * (int)cv.w;
    const int tap = k / (int)cv.cin, c = k - tap * (int)cv.cin;
    const int ty = tap / 3, tx = tap - 3 * ty;
    const int ys = y + ty - 1, xs = x + tx - 1;
    if ((unsigned)ys >= (unsigned)cv.lh || (unsigned)xs >= (unsigned)cv.lw) return 0.f;
    return src[(((long)b * cv.hs + (ys >> cv.sh)) * cv.ws + (xs >> cv.sh)) * ld + c];
  }
};

template <int AM, int BMD>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const EncdiffGemmArgs p, const F32Conv cv) {
  __shared__ float As[FBK][FBM + 4];
  __shared__ float Bs[FBK][FBN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * FBM, n0 = blockIdx.y * FBN;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const float* A = (const float*)p.a;
  const float* Bw = (const float*)p.b;
  const Im2F32 ia{A, p.conv.ld_src, cv}, ib{Bw, p.conv.ld_src, cv};
  // float4 staging (the forward forms): thread -> (row, 4 consecutive k)
  constexpr bool VEC = (AM == ENCDIFF_OPA_ROWK || AM == ENCDIFF_OPA_IM2COL) && BMD == ENCDIFF_OPB_ROWK;
  const int lr = tid >> 2, lk = (tid & 3) * 4;
  const int am = m0 + lr, bn = n0 + lr;
  int ab = 0, ay = 0, ax = 0;
  if (VEC && AM == ENCDIFF_OPA_IM2COL && am < p.M) {
    ab = am / (int)cv.hw;
    const int r = am - ab * (int)cv.hw;
    ay = r / (int)cv.w;
    ax = r - ay * (int)cv.w;
  }
  const bool bgrad = AM == ENCDIFF_OPA_ROWM && p.bias_grad && blockIdx.y == 0;
  float bsum = 0.f;
  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < p.K; k0 += FBK) {
    if constexpr (VEC) {
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
    } else {
      // generic element staging: thread -> (k row, m / n column), 4 elements of each operand
      float av[4], bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + 256 * j, kk = e >> 6, mm = e & 63;
        const int k = k0 + kk, m = m0 + mm, n = n0 + mm;
        float a = 0.f, b = 0.f;
        if (k < p.K && m < p.M) {
          if (AM == ENCDIFF_OPA_ROWK) a = A[(long)m * p.lda + k];
          else if (AM == ENCDIFF_OPA_ROWM) a = A[(long)k * p.lda + m];
          else a = ia.at(m, k);
        }
        if (k < p.K && n < p.N) {
          if (BMD == ENCDIFF_OPB_ROWK) b = Bw[(long)n * p.ldb + k];
          else if (BMD == ENCDIFF_OPB_ROWN) b = Bw[(long)k * p.ldb + n];
          else if (BMD == ENCDIFF_OPB_IM2COL) b = ib.at(k, n);
          else {  // CONV_DGRAD
            const int tap = k / p.conv_cout, co = k - tap * p.conv_cout;
            b = Bw[(long)co * p.ldb + (long)(8 - tap) * p.N + n];
          }
        }
        av[j] = a;
        bv[j] = b;
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = tid + 256 * j;
        As[e >> 6][e & 63] = av[j];
        Bs[e >> 6][e & 63] = bv[j];
      }
      __syncthreads();
      if (bgrad && tid < FBM) {
#pragma unroll
        for (int kk = 0; kk < FBK; ++kk) bsum += As[kk][tid];
      }
    }
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
  if (bgrad && tid < FBM && m0 + tid < p.M) p.bias_grad[m0 + tid] += bsum;
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

// ---------------------------------------------------------------- fp32 backward
ED_DEV float sig_f32(float z) { return 1.f / (1.f + expf(-z)); }
ED_DEV float silu_grad_f32(float z) {
  const float g = sig_f32(z);
  return g * (1.f + z * (1.f - g));
}
ED_DEV float gelu_grad_f32(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.39894228040143268f * expf(-0.5f * x * x);
}

// GroupNorm (+FiLM)(+SiLU) backward, one workgroup per (image, group), from the forward's saved
// (mean, rstd): u = (x^ gamma + beta)(1 + s) + sh, y = silu(u).  Per channel: d beta = sum dh,
// d gamma = sum dh x^ (per-image partials), d shift = sum du, d scale = sum du h; dx =
// rstd (dx^ - mean(dx^) - x^ mean(dx^ x^)) with dx^ = dh gamma (+ resid, or += into dx).
// Per-channel sums: a fixed thread -> channel map, partials added in thread order (reproducible).
__global__ __launch_bounds__(256) void gn_bwd_f32_kernel(const EncdiffGroupNormArgs p) {
  __shared__ float red[4][256];
  __shared__ float grp[2][4];
  const int b = blockIdx.x / p.groups, g = blockIdx.x - b * p.groups;
  const int cpg = p.c / p.groups, n = cpg * p.hw;
  const int tpc = 256 / cpg, nthr = tpc * cpg;  // threads per channel, active threads
  const int t = threadIdx.x, cl = t % cpg, c = g * cpg + cl;
  const float mean = p.stats[2 * blockIdx.x], rstd = p.stats[2 * blockIdx.x + 1];
  const float* X = (const float*)p.x + (long)b * p.hw * p.ldx + g * cpg;
  const float* DY = (const float*)p.dy + (long)b * p.hw * p.lddy + g * cpg;
  float gam = 0.f, bet = 0.f, sc = 0.f;
  if (t < nthr) {
    gam = p.gamma[c];
    bet = p.beta[c];
    if (p.film) sc = p.film[(long)b * p.ld_film + c];
  }
  const float sh = (t < nthr && p.film) ? p.film[(long)b * p.ld_film + p.c + c] : 0.f;
  float s_db = 0.f, s_dg = 0.f, s_dsh = 0.f, s_dsc = 0.f, s1 = 0.f, s2 = 0.f;
  if (t < nthr) {
    for (int px = t / cpg; px < p.hw; px += tpc) {
      const float xh = (X[(long)px * p.ldx + cl] - mean) * rstd;
      const float h = xh * gam + bet;
      const float u = p.film ? h * (1.f + sc) + sh : h;
      const float dy = DY[(long)px * p.lddy + cl];
      const float du = p.silu ? dy * silu_grad_f32(u) : dy;
      const float dh = p.film ? du * (1.f + sc) : du;
      const float dxh = dh * gam;
      s_db += dh;
      s_dg += dh * xh;
      s_dsh += du;
      s_dsc += du * h;
      s1 += dxh;
      s2 += dxh * xh;
    }
  }
  // group sums (block reduction, fixed order)
  float a1 = wave_sum(s1), a2 = wave_sum(s2);
  if ((t & 63) == 0) { grp[0][t >> 6] = a1; grp[1][t >> 6] = a2; }
  red[0][t] = s_db; red[1][t] = s_dg; red[2][t] = s_dsh; red[3][t] = s_dsc;
  __syncthreads();
  const float S1 = ((grp[0][0] + grp[0][1]) + grp[0][2]) + grp[0][3];
  const float S2 = ((grp[1][0] + grp[1][1]) + grp[1][2]) + grp[1][3];
  if (t < cpg) {
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    for (int j = t; j < nthr; j += cpg)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] += red[q][j];
    if (p.dbeta_part) p.dbeta_part[(long)b * p.ld_part + c] = v[0];
    if (p.dgamma_part) p.dgamma_part[(long)b * p.ld_part + c] = v[1];
    if (p.dfilm) {
      p.dfilm[(long)b * p.ld_dfilm + c] = v[3];
      p.dfilm[(long)b * p.ld_dfilm + p.c + c] = v[2];
    }
  }
  const float m1 = S1 / (float)n, m2 = S2 / (float)n;
  float* DX = (float*)p.dx + (long)b * p.hw * p.lddx + g * cpg;
  const float* RS = (const float*)p.resid;
  for (int i = t; i < n; i += 256) {
    const int px = i / cpg, cc = i - px * cpg, ch = g * cpg + cc;
    const float xh = (X[(long)px * p.ldx + cc] - mean) * rstd;
    const float h = xh * p.gamma[ch] + p.beta[ch];
    const float s_ = p.film ? p.film[(long)b * p.ld_film + ch] : 0.f;
    const float u = p.film ? h * (1.f + s_) + p.film[(long)b * p.ld_film + p.c + ch] : h;
    const float dy = DY[(long)px * p.lddy + cc];
    const float du = p.silu ? dy * silu_grad_f32(u) : dy;
    const float dxh = (p.film ? du * (1.f + s_) : du) * p.gamma[ch];
    float v = rstd * (dxh - m1 - xh * m2);
    if (RS) v += RS[((long)b * p.hw + px) * p.ld_resid + ch];
    float* dp = DX + (long)px * p.lddx + cc;
    *dp = p.accumulate_dx ? *dp + v : v;
  }
}

// LayerNorm backward over fp32 rows from the saved (mean, rstd): workgroup `part` owns a contiguous
// range of rows, one wave per row at a time; per-lane channel partials of d gamma / d beta, the 4
// waves' partials added in wave order -> dgamma_part[part][c].
__global__ __launch_bounds__(256) void ln_bwd_f32_kernel(const EncdiffLayerNormArgs p) {
  __shared__ float red[2][4][512];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int per = (p.rows + p.parts - 1) / p.parts;
  const int r0 = blockIdx.x * per, r1 = min(p.rows, r0 + per);
  constexpr int MAXJ = 8;  // c <= 512
  float dg[MAXJ], db[MAXJ];
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) dg[j] = db[j] = 0.f;
  const float* RS = (const float*)p.resid;
  for (int row = r0 + wave; row < r1; row += 4) {
    const float mean = p.stats[2L * row], rstd = p.stats[2L * row + 1];
    const float* X = (const float*)p.x + (long)row * p.ldx;
    const float* DY = (const float*)p.dy + (long)row * p.lddy;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < p.c) {
        const float xh = (X[c] - mean) * rstd, d = DY[c];
        const float gg = d * p.gamma[c];
        s1 += gg;
        s2 += gg * xh;
        dg[j] += d * xh;
        db[j] += d;
      }
    }
    const float m1 = wave_sum(s1) / (float)p.c, m2 = wave_sum(s2) / (float)p.c;
    float* DX = (float*)p.dx + (long)row * p.lddx;
#pragma unroll
    for (int j = 0; j < MAXJ; ++j) {
      const int c = lane + 64 * j;
      if (c < p.c) {
        const float xh = (X[c] - mean) * rstd;
        float v = rstd * (DY[c] * p.gamma[c] - m1 - xh * m2);
        if (RS) v += RS[(long)row * p.ld_resid + c];
        DX[c] = p.accumulate_dx ? DX[c] + v : v;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < MAXJ; ++j) {
    const int c = lane + 64 * j;
    if (c < 512) { red[0][wave][c] = dg[j]; red[1][wave][c] = db[j]; }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < p.c; c += 256) {
    if (p.dgamma_part)
      p.dgamma_part[(long)blockIdx.x * p.ld_part + c] = ((red[0][0][c] + red[0][1][c]) + red[0][2][c]) + red[0][3][c];
    if (p.dbeta_part)
      p.dbeta_part[(long)blockIdx.x * p.ld_part + c] = ((red[1][0][c] + red[1][1][c]) + red[1][2][c]) + red[1][3][c];
  }
}

// attention backward, exact fp32 from the saved log-sum-exp: P_ij = exp(s_ij - lse_i),
// dP_ij = dO_i . v_j, dS_ij = P_ij (dP_ij - D_i) with D_i = dO_i . O_i.
//   dq kernel : one thread per query, keys / values streamed through LDS; dq_i = scale sum_j dS_ij k_j
//   dkv kernel: one thread per key, queries / dO / D / lse streamed through LDS;
//               dv_j = sum_i P_ij dO_i, dk_j = scale sum_i dS_ij q_i
template <int DH>
__global__ __launch_bounds__(64) void attn_bwd_q_f32_kernel(const EncdiffAttnArgs p) {
  __shared__ float Ks[AKC][DH + 1];
  __shared__ float Vs[AKC][DH + 1];
  const int bh = blockIdx.y, b = bh / p.heads, h = bh - b * p.heads;
  const int qi = blockIdx.x * 64 + threadIdx.x;
  const bool live = qi < p.sq;
  const long qr = (long)b * p.sq + (live ? qi : 0);
  float q[DH], dq[DH], d_o[DH];
  float D = 0.f;
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    q[d] = ((const float*)p.q)[qr * p.ldq + h * DH + d];
    d_o[d] = ((const float*)p.d_o)[qr * p.lddo + h * DH + d];
    D += d_o[d] * ((const float*)p.o)[qr * p.ldo + h * DH + d];
    dq[d] = 0.f;
  }
  const float L = p.lse[(long)bh * p.sq + (live ? qi : 0)];
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
      float sc = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) { sc += q[d] * Ks[j][d]; dp += d_o[d] * Vs[j][d]; }
      const float pij = expf(sc * p.scale - L);
      const float ds = pij * (dp - D) * p.scale;
#pragma unroll
      for (int d = 0; d < DH; ++d) dq[d] += ds * Ks[j][d];
    }
  }
  if (!live) return;
  float* DQ = (float*)p.dq + qr * p.lddq + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) DQ[d] = dq[d];
}

constexpr int AQC = 64;
template <int DH>
__global__ __launch_bounds__(64) void attn_bwd_kv_f32_kernel(const EncdiffAttnArgs p) {
  __shared__ float Qs[AQC][DH + 1];
  __shared__ float Os[AQC][DH + 1];
  __shared__ float Ds[AQC], Ls[AQC];
  const int bh = blockIdx.y, b = bh / p.heads, h = bh - b * p.heads;
  const int kj = blockIdx.x * 64 + threadIdx.x;
  const bool live = kj < p.sk;
  const long kr = (long)b * p.sk + (live ? kj : 0);
  float k[DH], v[DH], dk[DH], dv[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    k[d] = ((const float*)p.k)[kr * p.ldk + h * DH + d];
    v[d] = ((const float*)p.v)[kr * p.ldv + h * DH + d];
    dk[d] = dv[d] = 0.f;
  }
  const float* Qg = (const float*)p.q + (long)b * p.sq * p.ldq + h * DH;
  const float* Og = (const float*)p.o + (long)b * p.sq * p.ldo + h * DH;
  const float* Gg = (const float*)p.d_o + (long)b * p.sq * p.lddo + h * DH;
  for (int q0 = 0; q0 < p.sq; q0 += AQC) {
    const int nq = min(AQC, p.sq - q0);
    __syncthreads();
    if (threadIdx.x < nq) {  // D_i = dO_i . O_i and lse_i of the chunk's queries
      float D = 0.f;
      for (int d = 0; d < DH; ++d) D += Gg[(long)(q0 + threadIdx.x) * p.lddo + d] * Og[(long)(q0 + threadIdx.x) * p.ldo + d];
      Ds[threadIdx.x] = D;
      Ls[threadIdx.x] = p.lse[(long)bh * p.sq + q0 + threadIdx.x];
    }
    for (int i = threadIdx.x; i < nq * DH; i += 64) {
      const int r = i / DH, d = i - r * DH;
      Qs[r][d] = Qg[(long)(q0 + r) * p.ldq + d];
      Os[r][d] = Gg[(long)(q0 + r) * p.lddo + d];  // dO rows
    }
    __syncthreads();
    for (int i = 0; i < nq; ++i) {
      float sc = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) { sc += Qs[i][d] * k[d]; dp += Os[i][d] * v[d]; }
      const float pij = expf(sc * p.scale - Ls[i]);
      const float ds = pij * (dp - Ds[i]) * p.scale;
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        dv[d] += pij * Os[i][d];
        dk[d] += ds * Qs[i][d];
      }
    }
  }
  if (!live) return;
  float* DK = (float*)p.dk + kr * p.lddk + h * DH;
  float* DV = (float*)p.dv + kr * p.lddv + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) { DK[d] = dk[d]; DV[d] = dv[d]; }
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
      case ENCDIFF_EW_SILU_BWD: v = X2[(long)r * p.ldx2 + c] * silu_grad_f32(X[(long)r * p.ldx + c]); break;
      case ENCDIFF_EW_GEGLU_BWD: {  // x: [rows][2*cols] proj output, x2 = dy; y[:, c], y[:, cols + c]
        const float a = X[(long)r * p.ldx + c], g = X[(long)r * p.ldx + p.cols + c];
        const float d = X2[(long)r * p.ldx2 + c];
        float* yp = Y + (long)r * p.ldy;
        const float da = d * (0.5f * g * (1.f + erff(g * 0.70710678118654752f))), dg = d * a * gelu_grad_f32(g);
        yp[c] = p.accumulate ? yp[c] + da : da;
        yp[p.cols + c] = p.accumulate ? yp[p.cols + c] + dg : dg;
        continue;
      }
      case ENCDIFF_EW_RESAMPLE_BWD: {  // adjoint; output (h, w) = the forward's source dims
        const int hw = p.h * p.w, b = r / hw, rr = r - b * hw, y = rr / p.w, x = rr - y * p.w;
        if (p.resample == ENCDIFF_RESAMPLE_DOWN2) {  // fwd avgpool (h, w) -> (h/2, w/2)
          v = 0.25f * X[(((long)b * (p.h >> 1) + (y >> 1)) * (p.w >> 1) + (x >> 1)) * p.ldx + c];
        } else {  // fwd nearest (h, w) -> (2h, 2w): the 4 children
          const int W2 = 2 * p.w;
          const long s0 = ((long)b * 2 * p.h + 2 * y) * W2 + 2 * x;
          v = (X[s0 * p.ldx + c] + X[(s0 + 1) * p.ldx + c]) + (X[(s0 + W2) * p.ldx + c] + X[(s0 + W2 + 1) * p.ldx + c]);
        }
        break;
      }
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
  if (p->M <= 0 || p->N <= 0 || p->K <= 0) return ENCDIFF_ERR_SHAPE;
  const int am = p->a_mode, bm = p->b_mode;
  if (am != ENCDIFF_OPA_ROWK && am != ENCDIFF_OPA_ROWM && am != ENCDIFF_OPA_IM2COL) return ENCDIFF_ERR_UNSUPPORTED;
  if (bm != ENCDIFF_OPB_ROWK && bm != ENCDIFF_OPB_ROWN && bm != ENCDIFF_OPB_IM2COL && bm != ENCDIFF_OPB_CONV_DGRAD)
    return ENCDIFF_ERR_UNSUPPORTED;
  if (am == ENCDIFF_OPA_IM2COL && bm == ENCDIFF_OPB_IM2COL) return ENCDIFF_ERR_UNSUPPORTED;
  if ((p->c_mode != ENCDIFF_OUT_F32 && p->c_mode != ENCDIFF_OUT_F32_ACCUM) || p->split_k > 1 || p->gn_stats || p->ln_y)
    return ENCDIFF_ERR_UNSUPPORTED;
  if (p->bias_grad && am != ENCDIFF_OPA_ROWM) return ENCDIFF_ERR_UNSUPPORTED;
  const bool vec = (am == ENCDIFF_OPA_ROWK || am == ENCDIFF_OPA_IM2COL) && bm == ENCDIFF_OPB_ROWK;
  if (vec && (p->K % 4 || p->lda % 4 || p->ldb % 4 || ((uintptr_t)p->a & 15) || ((uintptr_t)p->b & 15)))
    return ENCDIFF_ERR_SHAPE;
  F32Conv cv{};
  if (am == ENCDIFF_OPA_IM2COL || bm == ENCDIFF_OPB_IM2COL) {
    const int rs = p->conv.resample;
    if (rs != ENCDIFF_RESAMPLE_NONE && rs != ENCDIFF_RESAMPLE_UP2) return ENCDIFF_ERR_UNSUPPORTED;
    const long pix = (long)p->conv.batch * p->conv.h * p->conv.w;
    if (am == ENCDIFF_OPA_IM2COL && (p->K != 9 * p->conv.cin || p->M != pix)) return ENCDIFF_ERR_SHAPE;
    if (bm == ENCDIFF_OPB_IM2COL && (p->N != 9 * p->conv.cin || p->K != pix)) return ENCDIFF_ERR_SHAPE;
    if (vec && (p->conv.cin % 4 || p->conv.ld_src % 4)) return ENCDIFF_ERR_SHAPE;
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
  if (bm == ENCDIFF_OPB_CONV_DGRAD && (p->conv_cout <= 0 || p->K != 9 * p->conv_cout)) return ENCDIFF_ERR_SHAPE;
  dim3 grid((p->M + FBM - 1) / FBM, (p->N + FBN - 1) / FBN);
#define ED_F32_GEMM(AM_, BM_) \
  if (am == AM_ && bm == BM_) { hipLaunchKernelGGL((gemm_f32_kernel<AM_, BM_>), grid, dim3(256), 0, s, *p, cv); ED_CHECK_LAUNCH(); return ENCDIFF_OK; }
  ED_F32_GEMM(ENCDIFF_OPA_ROWK, ENCDIFF_OPB_ROWK)
  ED_F32_GEMM(ENCDIFF_OPA_IM2COL, ENCDIFF_OPB_ROWK)
  ED_F32_GEMM(ENCDIFF_OPA_ROWK, ENCDIFF_OPB_ROWN)
  ED_F32_GEMM(ENCDIFF_OPA_ROWM, ENCDIFF_OPB_ROWN)
  ED_F32_GEMM(ENCDIFF_OPA_ROWM, ENCDIFF_OPB_IM2COL)
  ED_F32_GEMM(ENCDIFF_OPA_IM2COL, ENCDIFF_OPB_CONV_DGRAD)
#undef ED_F32_GEMM
  return ENCDIFF_ERR_UNSUPPORTED;
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
  const int op = a->op;
  if (op != ENCDIFF_EW_COPY && op != ENCDIFF_EW_SILU && op != ENCDIFF_EW_GEGLU && op != ENCDIFF_EW_ADD &&
      op != ENCDIFF_EW_RESAMPLE && op != ENCDIFF_EW_SILU_BWD && op != ENCDIFF_EW_GEGLU_BWD &&
      op != ENCDIFF_EW_RESAMPLE_BWD)
    return ENCDIFF_ERR_UNSUPPORTED;
  if ((op == ENCDIFF_EW_ADD || op == ENCDIFF_EW_SILU_BWD || op == ENCDIFF_EW_GEGLU_BWD) && !a->x2) return ENCDIFF_ERR_ARG;
  if ((op == ENCDIFF_EW_RESAMPLE || op == ENCDIFF_EW_RESAMPLE_BWD) && a->resample != ENCDIFF_RESAMPLE_DOWN2 &&
      a->resample != ENCDIFF_RESAMPLE_UP2)
    return ENCDIFF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(ew_f32_kernel, dim3(grid256((long)a->rows * a->cols)), dim3(256), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_groupnorm_bwd_f32(const EncdiffGroupNormArgs* a, hipStream_t s) {
  if (!a->x || !a->dy || !a->dx || !a->stats || !a->gamma || !a->beta) return ENCDIFF_ERR_ARG;
  if (a->groups <= 0 || a->c % a->groups || a->c / a->groups > 256 || a->in_stats || a->x_from)
    return ENCDIFF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(gn_bwd_f32_kernel, dim3(a->batch * a->groups), dim3(256), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_layernorm_bwd_f32(const EncdiffLayerNormArgs* a, hipStream_t s) {
  if (!a->x || !a->dy || !a->dx || !a->stats || !a->gamma || a->parts <= 0) return ENCDIFF_ERR_ARG;
  if (a->c > 512 || a->dy_from) return ENCDIFF_ERR_UNSUPPORTED;
  hipLaunchKernelGGL(ln_bwd_f32_kernel, dim3(a->parts), dim3(256), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int ed_attention_bwd_f32(const EncdiffAttnArgs* a, hipStream_t s) {
  if (!a->q || !a->k || !a->v || !a->o || !a->lse || !a->d_o || !a->dq || !a->dk || !a->dv || a->fp8_qk)
    return ENCDIFF_ERR_ARG;
  dim3 gq((a->sq + 63) / 64, a->batch * a->heads), gk((a->sk + 63) / 64, a->batch * a->heads);
  switch (a->dh) {
#define ED_ATTN_BWD_F32(D)                                                          \
    case D:                                                                         \
      hipLaunchKernelGGL(attn_bwd_q_f32_kernel<D>, gq, dim3(64), 0, s, *a);         \
      hipLaunchKernelGGL(attn_bwd_kv_f32_kernel<D>, gk, dim3(64), 0, s, *a);        \
      break;
    ED_ATTN_BWD_F32(8)
    ED_ATTN_BWD_F32(16)
    ED_ATTN_BWD_F32(32)
    ED_ATTN_BWD_F32(64)
#undef ED_ATTN_BWD_F32
    default: return ENCDIFF_ERR_SHAPE;
  }
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
