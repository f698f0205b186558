// norm.hip -- GroupNorm(+FiLM)(+SiLU) and LayerNorm, forward and backward, NHWC bf16.
//
// GroupNorm: one workgroup per image (512 threads).  Threads are laid out as
// (C/8 channel vectors) x (pixel lanes); each thread streams 16-byte vectors of its
// 8 channels over its pixels, sums are combined through LDS into per-channel and
// per-group statistics (fp32, as GroupNorm32 does: util.py:242-244), then a second
// pass (L2-resident re-read) writes the normalised, FiLM-modulated, SiLU-activated
// output (openaimodel_enc.py:201-205, 225-232, 267-271, 684-686; attention.py:76-77).
// The backward recomputes the forward from x and the saved statistics and emits
// per-image partial sums for dgamma/dbeta (reduced once per step by
// encdiff_reduce_partials) and the FiLM gradients d(scale), d(shift) per (b, c).
#include "common.h"

namespace {

constexpr int GN_THREADS = 512;

struct GnLayout {
  int nv, np, tv, tp;
  ED_DEV GnLayout(int c) {
    nv = c >> 3;
    np = GN_THREADS / nv;
    while (np & (np - 1)) np &= np - 1;  // power-of-two pixel lanes (tree reduction)
    tv = threadIdx.x % nv;
    tp = threadIdx.x / nv;
  }
};

// Tree-reduce NR arrays red[k][np][C] over the np rows into row 0 (log2(np) steps).
// Every thread of the block must call it.
ED_DEV void tree_reduce_rows(float* red, int NR, const GnLayout& L, int C) {
  for (int stride = L.np >> 1; stride > 0; stride >>= 1) {
    __syncthreads();
    if (L.tp < stride) {
      for (int k = 0; k < NR; ++k) {
        float4* a = (float4*)(red + (k * L.np + L.tp) * C + L.tv * 8);
        const float4* b = (const float4*)(red + (k * L.np + L.tp + stride) * C + L.tv * 8);
        float4 a0 = a[0], a1 = a[1];
        const float4 b0 = b[0], b1 = b[1];
        a0.x += b0.x; a0.y += b0.y; a0.z += b0.z; a0.w += b0.w;
        a1.x += b1.x; a1.y += b1.y; a1.z += b1.z; a1.w += b1.w;
        a[0] = a0; a[1] = a1;
      }
    }
  }
  __syncthreads();
}

__global__ __launch_bounds__(GN_THREADS) void gn_fwd_kernel(const EncdiffGroupNormArgs p) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int b = blockIdx.x;
  const int C = p.c, HW = p.hw, cpg = C / p.groups;
  GnLayout L(C);
  float* red = sh;                      // [np][C] x2
  float* ch_s = sh + 2 * L.np * C;      // [C]
  float* ch_ss = ch_s + C;              // [C]
  float* g_mean = ch_ss + C;            // [groups]
  float* g_rstd = g_mean + p.groups;    // [groups]

  const bf16_t* X = (const bf16_t*)p.x + (long)b * HW * p.ldx;
  const bool active = L.tp < L.np;
  float s[8], ss[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { s[i] = 0.f; ss[i] = 0.f; }
  if (active) {
    for (int px = L.tp; px < HW; px += L.np) {
      float v[8];
      unpack8(*(const uint4*)(X + (long)px * p.ldx + L.tv * 8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += v[i]; ss[i] += v[i] * v[i]; }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[L.tp * C + L.tv * 8 + i] = s[i];
      red[(L.np + L.tp) * C + L.tv * 8 + i] = ss[i];
    }
  }
  tree_reduce_rows(red, 2, L, C);
  for (int c = threadIdx.x; c < C; c += GN_THREADS) {
    ch_s[c] = red[c];
    ch_ss[c] = red[L.np * C + c];
  }
  __syncthreads();
  if (threadIdx.x < p.groups) {
    const int g = threadIdx.x;
    float a = 0.f, q = 0.f;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) { a += ch_s[c]; q += ch_ss[c]; }
    const float n = (float)HW * cpg;
    const float mean = a / n;
    const float var = fmaxf(q / n - mean * mean, 0.f);
    const float rstd = rsqrtf(var + p.eps);
    g_mean[g] = mean; g_rstd[g] = rstd;
    p.stats[(b * p.groups + g) * 2] = mean;
    p.stats[(b * p.groups + g) * 2 + 1] = rstd;
  }
  __syncthreads();
  if (!active) return;
  // per-thread channel constants
  float mul[8], add[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = L.tv * 8 + i;
    const int g = c / cpg;
    float ga = p.gamma[c], be = p.beta[c];
    float m = g_mean[g], r = g_rstd[g];
    // y = ((x - m) r ga + be)(1 + sc) + sh
    float a = r * ga, bb = be - m * r * ga;
    if (p.film) {
      const float sc = p.film[(long)b * p.ld_film + c];
      const float sf = p.film[(long)b * p.ld_film + C + c];
      a *= (1.f + sc);
      bb = bb * (1.f + sc) + sf;
    }
    mul[i] = a; add[i] = bb;
  }
  bf16_t* Y = (bf16_t*)p.y + (long)b * HW * p.ldy;
  for (int px = L.tp; px < HW; px += L.np) {
    float v[8];
    unpack8(*(const uint4*)(X + (long)px * p.ldx + L.tv * 8), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float z = v[i] * mul[i] + add[i];
      v[i] = p.silu ? silu_f(z) : z;
    }
    *(uint4*)(Y + (long)px * p.ldy + L.tv * 8) = pack8(v);
  }
}

__global__ __launch_bounds__(GN_THREADS) void gn_bwd_kernel(const EncdiffGroupNormArgs p) {
  extern __shared__ __attribute__((aligned(16))) float sh[];
  const int b = blockIdx.x;
  const int C = p.c, HW = p.hw, cpg = C / p.groups;
  GnLayout L(C);
  const bool film = p.film != nullptr;
  const int NR = film ? 4 : 2;           // reductions per channel
  float* red = sh;                       // [NR][np][C]
  float* chs = sh + NR * L.np * C;       // [NR][C]
  float* gs = chs + NR * C;              // [groups][2]
  const float* st = p.stats + b * p.groups * 2;

  const bf16_t* X = (const bf16_t*)p.x + (long)b * HW * p.ldx;
  const bf16_t* DY = (const bf16_t*)p.dy + (long)b * HW * p.lddy;
  const bool active = L.tp < L.np;

  float xm[8], xr[8], ga[8], be[8], sc1[8], sf[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = L.tv * 8 + i;
    const int g = c / cpg;
    xm[i] = st[2 * g]; xr[i] = st[2 * g + 1];
    ga[i] = p.gamma[c]; be[i] = p.beta[c];
    sc1[i] = film ? 1.f + p.film[(long)b * p.ld_film + c] : 1.f;
    sf[i] = film ? p.film[(long)b * p.ld_film + C + c] : 0.f;
  }
  // pass 1: per-channel sums of dn, dn*xhat (and dz, dz*n for FiLM)
  float a_dn[8], a_dnx[8], a_dz[8], a_dzn[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { a_dn[i] = a_dnx[i] = a_dz[i] = a_dzn[i] = 0.f; }
  if (active) {
    for (int px = L.tp; px < HW; px += L.np) {
      float v[8], d[8];
      unpack8(*(const uint4*)(X + (long)px * p.ldx + L.tv * 8), v);
      unpack8(*(const uint4*)(DY + (long)px * p.lddy + L.tv * 8), d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (v[i] - xm[i]) * xr[i];
        const float n = xh * ga[i] + be[i];
        const float z = n * sc1[i] + sf[i];
        const float dz = p.silu ? d[i] * silu_grad(z) : d[i];
        const float dn = dz * sc1[i];
        a_dn[i] += dn; a_dnx[i] += dn * xh;
        a_dz[i] += dz; a_dzn[i] += dz * n;
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int c = L.tv * 8 + i;
      red[(0 * L.np + L.tp) * C + c] = a_dn[i];
      red[(1 * L.np + L.tp) * C + c] = a_dnx[i];
      if (film) {
        red[(2 * L.np + L.tp) * C + c] = a_dz[i];
        red[(3 * L.np + L.tp) * C + c] = a_dzn[i];
      }
    }
  }
  tree_reduce_rows(red, NR, L, C);
  for (int c = threadIdx.x; c < C; c += GN_THREADS) {
    for (int k = 0; k < NR; ++k) chs[k * C + c] = red[(k * L.np) * C + c];
    p.dbeta_part[(long)b * p.ld_part + c] = chs[c];
    p.dgamma_part[(long)b * p.ld_part + c] = chs[C + c];
    if (film) {
      p.dfilm[(long)b * p.ld_dfilm + c] = chs[3 * C + c];       // d scale = sum dz * n
      p.dfilm[(long)b * p.ld_dfilm + C + c] = chs[2 * C + c];   // d shift = sum dz
    }
  }
  __syncthreads();
  if (threadIdx.x < p.groups) {
    const int g = threadIdx.x;
    float s1 = 0.f, s2 = 0.f;
    for (int c = g * cpg; c < (g + 1) * cpg; ++c) {
      s1 += p.gamma[c] * chs[c];
      s2 += p.gamma[c] * chs[C + c];
    }
    const float inv_n = 1.f / ((float)HW * cpg);
    gs[2 * g] = s1 * inv_n;
    gs[2 * g + 1] = s2 * inv_n;
  }
  __syncthreads();
  if (!active) return;
  float m1[8], m2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = (L.tv * 8 + i) / cpg;
    m1[i] = gs[2 * g]; m2[i] = gs[2 * g + 1];
  }
  bf16_t* DX = (bf16_t*)p.dx + (long)b * HW * p.lddx;
  for (int px = L.tp; px < HW; px += L.np) {
    float v[8], d[8];
    unpack8(*(const uint4*)(X + (long)px * p.ldx + L.tv * 8), v);
    unpack8(*(const uint4*)(DY + (long)px * p.lddy + L.tv * 8), d);
    float o[8];
    if (p.accumulate_dx) unpack8(*(const uint4*)(DX + (long)px * p.lddx + L.tv * 8), o);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xh = (v[i] - xm[i]) * xr[i];
      const float n = xh * ga[i] + be[i];
      const float z = n * sc1[i] + sf[i];
      const float dz = p.silu ? d[i] * silu_grad(z) : d[i];
      const float dn = dz * sc1[i];
      const float r = xr[i] * (dn * ga[i] - m1[i] - xh * m2[i]);
      o[i] = p.accumulate_dx ? o[i] + r : r;
    }
    *(uint4*)(DX + (long)px * p.lddx + L.tv * 8) = pack8(o);
  }
}

// ---------------------------------------------------------------- LayerNorm
// A row of C channels is owned by C/8 lanes (8 channels per lane); 256 threads.
template <int C>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const EncdiffLayerNormArgs p) {
  constexpr int LPR = C / 8;               // lanes per row
  constexpr int RPB = 256 / LPR;           // rows per block-iteration
  const int lr = threadIdx.x % LPR;
  const int rr = threadIdx.x / LPR;
  float ga[8], be[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { ga[i] = p.gamma[lr * 8 + i]; be[i] = p.beta[lr * 8 + i]; }
  for (int row = blockIdx.x * RPB + rr; row < p.rows; row += gridDim.x * RPB) {
    float v[8];
    unpack8(*(const uint4*)((const bf16_t*)p.x + (long)row * p.ldx + lr * 8), v);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += v[i];
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.f / C);
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) { const float d = v[i] - mean; q += d * d; }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) q += __shfl_xor(q, o, 64);
    const float rstd = rsqrtf(q * (1.f / C) + p.eps);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (v[i] - mean) * rstd * ga[i] + be[i];
    *(uint4*)((bf16_t*)p.y + (long)row * p.ldy + lr * 8) = pack8(v);
    if (lr == 0) { p.stats[2 * row] = mean; p.stats[2 * row + 1] = rstd; }
  }
}

template <int C>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const EncdiffLayerNormArgs p) {
  constexpr int LPR = C / 8;
  constexpr int RPB = 256 / LPR;
  __shared__ float red[2][RPB][C];
  const int lr = threadIdx.x % LPR;
  const int rr = threadIdx.x / LPR;
  float ga[8], dga[8], dbe[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { ga[i] = p.gamma[lr * 8 + i]; dga[i] = 0.f; dbe[i] = 0.f; }
  for (int row = blockIdx.x * RPB + rr; row < p.rows; row += gridDim.x * RPB) {
    float v[8], d[8];
    unpack8(*(const uint4*)((const bf16_t*)p.x + (long)row * p.ldx + lr * 8), v);
    unpack8(*(const uint4*)((const bf16_t*)p.dy + (long)row * p.lddy + lr * 8), d);
    const float mean = p.stats[2 * row], rstd = p.stats[2 * row + 1];
    float s1 = 0.f, s2 = 0.f, xh[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      xh[i] = (v[i] - mean) * rstd;
      const float g = d[i] * ga[i];
      s1 += g; s2 += g * xh[i];
      dga[i] += d[i] * xh[i];
      dbe[i] += d[i];
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
    s1 *= (1.f / C); s2 *= (1.f / C);
    bf16_t* dxp = (bf16_t*)p.dx + (long)row * p.lddx + lr * 8;
    float o8[8];
    if (p.accumulate_dx) unpack8(*(const uint4*)dxp, o8);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float r = rstd * (d[i] * ga[i] - s1 - xh[i] * s2);
      o8[i] = p.accumulate_dx ? o8[i] + r : r;
    }
    *(uint4*)dxp = pack8(o8);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) { red[0][rr][lr * 8 + i] = dga[i]; red[1][rr][lr * 8 + i] = dbe[i]; }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += 256) {
    float a = 0.f, bsum = 0.f;
    for (int r = 0; r < RPB; ++r) { a += red[0][r][c]; bsum += red[1][r][c]; }
    p.dgamma_part[(long)blockIdx.x * p.ld_part + c] = a;
    p.dbeta_part[(long)blockIdx.x * p.ld_part + c] = bsum;
  }
}

size_t gn_fwd_lds(int C, int groups) {
  const int np = GN_THREADS / (C / 8);
  return (2 * np * C + 2 * C + 2 * groups) * sizeof(float);
}
size_t gn_bwd_lds(int C, int groups, bool film) {
  const int np = GN_THREADS / (C / 8);
  const int NR = film ? 4 : 2;
  return (NR * np * C + NR * C + 2 * groups) * sizeof(float);
}

}  // namespace

extern "C" int encdiff_groupnorm_fwd(const EncdiffGroupNormArgs* a, void* stream) {
  if (!a || !a->x || !a->y || !a->stats || !a->gamma || !a->beta) return ENCDIFF_ERR_ARG;
  if (a->c % 8 || a->c % a->groups || a->c > 8 * GN_THREADS || a->groups > GN_THREADS) return ENCDIFF_ERR_SHAPE;
  const size_t lds = gn_fwd_lds(a->c, a->groups);
  static const hipError_t attr = hipFuncSetAttribute((const void*)gn_fwd_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  hipLaunchKernelGGL(gn_fwd_kernel, dim3(a->batch), dim3(GN_THREADS), lds, (hipStream_t)stream, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_groupnorm_bwd(const EncdiffGroupNormArgs* a, void* stream) {
  if (!a || !a->x || !a->dy || !a->dx || !a->stats || !a->dgamma_part || !a->dbeta_part) return ENCDIFF_ERR_ARG;
  if (a->film && !a->dfilm) return ENCDIFF_ERR_ARG;
  if (a->c % 8 || a->c % a->groups || a->c > 8 * GN_THREADS || a->groups > GN_THREADS) return ENCDIFF_ERR_SHAPE;
  const size_t lds = gn_bwd_lds(a->c, a->groups, a->film != nullptr);
  static const hipError_t attr = hipFuncSetAttribute((const void*)gn_bwd_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  hipLaunchKernelGGL(gn_bwd_kernel, dim3(a->batch), dim3(GN_THREADS), lds, (hipStream_t)stream, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

template <int C>
static int ln_launch(const EncdiffLayerNormArgs& a, bool bwd, hipStream_t s) {
  constexpr int RPB = 256 / (C / 8);
  if (bwd) {
    hipLaunchKernelGGL(ln_bwd_kernel<C>, dim3(a.parts), dim3(256), 0, s, a);
  } else {
    int grid = (a.rows + RPB - 1) / RPB;
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(ln_fwd_kernel<C>, dim3(grid), dim3(256), 0, s, a);
  }
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

static int ln_dispatch(const EncdiffLayerNormArgs* a, bool bwd, void* stream) {
  if (!a) return ENCDIFF_ERR_ARG;
  if (bwd && (a->parts <= 0 || !a->dgamma_part || !a->dbeta_part || !a->dy || !a->dx)) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  switch (a->c) {
    case 64: return ln_launch<64>(*a, bwd, s);
    case 128: return ln_launch<128>(*a, bwd, s);
    case 256: return ln_launch<256>(*a, bwd, s);
    case 512: return ln_launch<512>(*a, bwd, s);
    default: return ENCDIFF_ERR_UNSUPPORTED;
  }
}

extern "C" int encdiff_layernorm_fwd(const EncdiffLayerNormArgs* a, void* stream) { return ln_dispatch(a, false, stream); }
extern "C" int encdiff_layernorm_bwd(const EncdiffLayerNormArgs* a, void* stream) { return ln_dispatch(a, true, stream); }
