// st_common.h -- device helpers shared by the SpatialTransformer row-tile kernels (st_fused.hip:
// forward head / tail; st_bwd.hip: their backward): weight fragments streamed from L2 into MFMA B
// operands, 16-row MFMA tiles over LDS rows, LayerNorm over LDS rows, row copies.
#pragma once
#include "common.h"

namespace {

typedef __bf16 v2bf_t __attribute__((ext_vector_type(2)));
// c + a.lo * b.lo + a.hi * b.hi over bf16 pairs as stored (v_dot2_f32_bf16: the exact products,
// fp32 accumulation)
ED_DEV float dot2bf(unsigned a, unsigned b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(v2bf_t, a), __builtin_bit_cast(v2bf_t, b), c, false);
}

// GELU (erf form, F.gelu's default) with a branch-free erf: Abramowitz-Stegun 7.1.26, |error| <=
// 1.5e-7 -- far below the bf16 rounding of a -- instead of ocml erff's range branches, which made
// the GEGLU chunk the tail kernel's longest stage.
ED_DEV float gelu_fast(float x) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float erf_abs = 1.f - poly * __expf(-z * z);
  return 0.5f * x * (1.f + copysignf(erf_abs, x));
}

// B fragments of W[n0 + 16 j + col][k0 + k] for k < K (lane: column l16, k = kk*32 + g4*8 .. +8)
template <int NT, int K>
struct BFrags {
  v8bf f[K / 32][NT];
};
template <int NT, int K>
ED_DEV void load_b(BFrags<NT, K>& b, const bf16_t* __restrict__ W, long ldw, int n0, int k0, int lane) {
  const int l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < K / 32; ++kk)
#pragma unroll
    for (int j = 0; j < NT; ++j)
      b.f[kk][j] = *(const v8bf*)(W + (long)(n0 + 16 * j + l16) * ldw + k0 + kk * 32 + g4 * 8);
}
// acc[i][j] += X[16 i + row][k] * B   (X in LDS, row stride ldx, k < K)
template <int TM, int NT, int K>
ED_DEV void mma(v4f (&acc)[TM][NT], const bf16_t* X, int ldx, const BFrags<NT, K>& b, int lane) {
  const int l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < K / 32; ++kk) {
    v8bf af[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) af[i] = *(const v8bf*)(X + (16 * i + l16) * ldx + kk * 32 + g4 * 8);
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], b.f[kk][j], acc[i][j], 0, 0, 0);
  }
}
template <int TM, int NT>
ED_DEV void zero(v4f (&acc)[TM][NT]) {
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
}
// accumulator element (i, j, q): row 16 i + 4 g4 + q, column n0 + 16 j + l16
template <int TM, int NT>
ED_DEV void acc_add_tr(const v4f (&acc)[TM][NT], float* Tr, int ldt, const float* __restrict__ bias, int n0, int lane) {
  const int l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = n0 + 16 * j + l16;
    const float bv = bias[col];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) Tr[(16 * i + 4 * g4 + q) * ldt + col] += acc[i][j][q] + bv;
  }
}
template <int TM, int NT>
ED_DEV void acc_store_bf(const v4f (&acc)[TM][NT], bf16_t* X, int ldx, int n0, int lane) {
  const int l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) X[(16 * i + 4 * g4 + q) * ldx + n0 + 16 * j + l16] = f2bf(acc[i][j][q]);
}

// LayerNorm of the R residual rows (fp32, LDS) into the bf16 operand buffer; optional saves.  The
// statistics are those of the bf16-rounded rows (the tensor the unfused path stores and its
// LayerNorm backward re-reads); the residual stream itself stays fp32.
template <int C, int R, int NTH = 256>
ED_DEV void ln_rows(const float* Tr, int ldt, bf16_t* X, int ldx, const float* __restrict__ g,
                    const float* __restrict__ b, float eps, int tid, bf16_t* save_y, long ld_save,
                    bf16_t* save_x, float* save_s) {
  // all R rows at once: TPR consecutive lanes per row, each owning float4 chunks k, k + TPR, ...
  // (a row per wave with 64-lane butterflies serialised R/4 rows of ds_bpermute round trips)
  constexpr int TPR = NTH / R, NQ = C / (4 * TPR);
  const int r = tid / TPR, k = tid % TPR;
  float v[NQ][4], s = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const float4 f = *(const float4*)(Tr + r * ldt + 4 * (k + TPR * i));
    // the stored (bf16) residual, as the unfused path normalises it
    v[i][0] = bf16_round(f.x); v[i][1] = bf16_round(f.y); v[i][2] = bf16_round(f.z); v[i][3] = bf16_round(f.w);
    s += (v[i][0] + v[i][1]) + (v[i][2] + v[i][3]);
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) s += __shfl_xor(s, o, 64);
  const float mean = s * (1.f / C);
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) s2 += (v[i][e] - mean) * (v[i][e] - mean);
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) s2 += __shfl_xor(s2, o, 64);
  const float rstd = rsqrtf(s2 * (1.f / C) + eps);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int c = 4 * (k + TPR * i);
    const float4 gv = make_float4(g[c], g[c + 1], g[c + 2], g[c + 3]);  // fp32 arena: 4-byte alignment only
    const float4 bv = make_float4(b[c], b[c + 1], b[c + 2], b[c + 3]);
    const uint2 y = make_uint2(pack2((v[i][0] - mean) * rstd * gv.x + bv.x, (v[i][1] - mean) * rstd * gv.y + bv.y),
                               pack2((v[i][2] - mean) * rstd * gv.z + bv.z, (v[i][3] - mean) * rstd * gv.w + bv.w));
    *(uint2*)(X + r * ldx + c) = y;
    if (save_y) {
      *(uint2*)(save_y + r * ld_save + c) = y;
      *(uint2*)(save_x + r * ld_save + c) = make_uint2(pack2(v[i][0], v[i][1]), pack2(v[i][2], v[i][3]));
    }
  }
  if (save_s && k == 0) {
    save_s[2 * r] = mean;
    save_s[2 * r + 1] = rstd;
  }
}

// copy R rows x C bf16 between global and LDS (16-byte chunks)
template <int C, int R, int NTH = 256>
ED_DEV void rows_to_lds(bf16_t* X, int ldx, const bf16_t* __restrict__ g, long ldg, int tid) {
  constexpr int CH = C / 8;
  for (int e = tid; e < R * CH; e += NTH) {
    const int r = e / CH, c8 = (e - r * CH) * 8;
    *(uint4*)(X + r * ldx + c8) = *(const uint4*)(g + (long)r * ldg + c8);
  }
}
template <int C, int R, int NTH = 256>
ED_DEV void rows_to_global(bf16_t* __restrict__ g, long ldg, const bf16_t* X, int ldx, int tid) {
  constexpr int CH = C / 8;
  for (int e = tid; e < R * CH; e += NTH) {
    const int r = e / CH, c8 = (e - r * CH) * 8;
    *(uint4*)(g + (long)r * ldg + c8) = *(const uint4*)(X + r * ldx + c8);
  }
}

}  // namespace
