// Shared device helpers for the EncDiff gfx950 kernels.
// All activations are NHWC / token-major bf16 ([rows][channels] with a row
// stride `ld` in elements); statistics and master weights are fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/encdiff_hip.h"

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));

#define ED_DEV __device__ __forceinline__

ED_DEV float bf2f(bf16_t u) { return __uint_as_float(((uint32_t)u) << 16); }
// Split-K combine epilogue alpha * sum (+ bias): ONE explicit FMA (bias 0 when absent), so every
// restatement of the combine (finalize pass, in-kernel fold, the GroupNorm / LayerNorm slab
// combines) rounds alike whatever -ffp-contract=fast does with the surrounding code -- that flag
// fuses across statements and ignores `#pragma clang fp contract`.  The residual is a plain add
// of this result (nothing left to contract).
ED_DEV float splitk_scale(float acc, float alpha, float bias) { return __builtin_fmaf(alpha, acc, bias); }
ED_DEV bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN preserving
  return __builtin_bit_cast(bf16_t, b);
}
typedef float v2f __attribute__((ext_vector_type(2)));
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 (two scalar conversions + a v_perm otherwise)
ED_DEV uint32_t pack2(float a, float b) {
  const v2f v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, v2bf));
}

// 8 bf16 <-> 8 float
ED_DEV void unpack8(const uint4& u, float* f) {
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
  }
}
ED_DEV uint4 pack8(const float* f) {
  uint4 u;
  u.x = pack2(f[0], f[1]); u.y = pack2(f[2], f[3]);
  u.z = pack2(f[4], f[5]); u.w = pack2(f[6], f[7]);
  return u;
}

// exact (erf) GELU, F.gelu's default (attention.py GEGLU)
ED_DEV float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
ED_DEV float gelu_erf_grad(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.39894228040143268f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}
ED_DEV float bf16_round(float x) { return bf2f(f2bf(x)); }

// sigmoid via the hardware reciprocal (v_rcp_f32, 1 ulp): results are rounded to bf16
ED_DEV float sigmoid_f(float z) { return __builtin_amdgcn_rcpf(1.0f + __expf(-z)); }
ED_DEV float silu_f(float z) { return z * sigmoid_f(z); }
ED_DEV float silu_grad(float z) {
  const float s = sigmoid_f(z);
  return s * (1.0f + z * (1.0f - s));
}
// SiLU(z) (bitwise silu_f) and, in g, silu_grad(z) from the one sigmoid
ED_DEV float silu_and_grad(float z, float& g) {
  const float s = sigmoid_f(z);
  g = s * (1.0f + z * (1.0f - s));
  return z * s;
}

ED_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Error codes of the C-ABI (see include/encdiff_hip.h)
#define ED_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)_e; \
  } while (0)

// fp32 (ENCDIFF_DT_F32) forms of the entry points, fp32.hip
int ed_gemm_f32(const EncdiffGemmArgs* p, hipStream_t s);
int ed_groupnorm_fwd_f32(const EncdiffGroupNormArgs* a, hipStream_t s);
int ed_layernorm_fwd_f32(const EncdiffLayerNormArgs* a, hipStream_t s);
int ed_attention_fwd_f32(const EncdiffAttnArgs* a, hipStream_t s);
int ed_elementwise_f32(const EncdiffEwArgs* a, hipStream_t s);
int ed_groupnorm_bwd_f32(const EncdiffGroupNormArgs* a, hipStream_t s);
int ed_layernorm_bwd_f32(const EncdiffLayerNormArgs* a, hipStream_t s);
int ed_attention_bwd_f32(const EncdiffAttnArgs* a, hipStream_t s);
