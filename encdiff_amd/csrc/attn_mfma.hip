// attn_mfma.hip -- MFMA attention for the SpatialTransformer heads (attention.py:170-193)
// and the VQ encoder's single-head AttnBlock (model.py:178-200, forward only).
//
// v_mfma_f32_16x16x16_bf16 (K = 16) tiles; head dims 8/16/32/64/128, 8 zero-padded to 16.
// Forward: per wave a pair of 16-query tiles; S^T = K Q^T is computed "swapped" so each lane
// holds 4 consecutive keys of ONE query: the row max of the online softmax is in-register plus
// two cross-lane xor-shuffles, and the bf16 P is already the B operand of O^T = V^T P^T (no
// LDS round trip for P).  K and V of the block's heads live in LDS row-major; the V^T operand
// is read transposed (ds_read_b64_tr_b16).
//
// The kernels are VALU-bound (exp / max / convert per score; the QK^T and PV MFMAs are a few
// percent of the issue slots even at dh = 8, where K is half padding), so the work per score is
// what is trimmed: the softmax scale is folded into the exp's FMA (max over raw scores), and at
// dh = 8 the softmax denominator comes out of the PV MFMA for free -- V^T's first padding row
// is all ones, so O^T row 8 accumulates sum_k p under the same online rescaling.
//
// Backward (recompute from LSE, no score matrix in HBM): phase A -- waves own key tiles and
// accumulate dK^T, dV^T over all query tiles, computing dS = P (dP - D); phase B -- waves own
// query tiles and accumulate dQ^T = K^T dS^T over all key tiles.  When a head group's dS fits
// the workgroup's LDS (S <= 256) phase A leaves dS^T there and phase B is MFMAs only (no
// second exp pass); otherwise phase B recomputes it.  Q, K, V, dO are staged row-major in LDS
// once per (image, head group) -- unpadded at dh = 8 -- the Q^T, K^T, dO^T operands are
// transposed reads of them, and rowsum(dO * O) is computed while staging.
//
// F8 (configs[4]'s S = 1024 level): the scores Q K^T come from v_mfma_f32_16x16x32_fp8_fp8
// on OCP e4m3 operands (Q, K rounded to e4m3; the same scores in the backward's recompute);
// softmax, P V and every gradient product stay bf16 / fp32.
#include "common.h"

// Built with -fno-honor-nans -mno-amdgpu-ieee (build.py): no v_max canonicalisation of MFMA
// results in the softmax max trees (scores are finite; masked keys are -inf, never NaN).

namespace {

typedef short s4 __attribute__((ext_vector_type(4)));

ED_DEV v4f mma(const s4& a, const s4& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
ED_DEV s4 ld4(const bf16_t* p) { return *(const s4*)p; }
// Transposed MFMA operand from a row-major LDS tile [rows][ld]: lane (l16, g) receives
// t[r0 + 4g + i][c0 + l16], i = 0..3 -- the A (or B) fragment whose k runs along the tile's
// rows -- via ds_read_b64_tr_b16: lane (tq, tp) = (l16 >> 2, l16 & 3) addresses row
// r0 + 4g + tq, columns c0 + 4tp .. +3.  Needs every lane of the wave active.  With a row pitch
// narrower than 16 (dh = 8 staging) lanes l16 >= 8 read the next row: those land in output rows
// (head-dim rows >= dh) that are never stored.
typedef __attribute__((address_space(3))) s4 lds_s4;
ED_DEV s4 ldtr(const bf16_t* t, int ld, int r0, int c0, int l16, int g) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(t + (r0 + 4 * g + (l16 >> 2)) * ld + c0 + 4 * (l16 & 3)));
}
ED_DEV s4 pack4(float a, float b, float c, float d) {
  const uint2 u = {pack2(a, b), pack2(c, d)};
  return __builtin_bit_cast(s4, u);
}

// ---- fp8 (OCP e4m3) score fragments: lane (g, l16) holds elements 8g .. 8g+7 of row l16 ----
ED_DEV v4f mma8(long a, long b, const v4f& c) { return __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(a, b, c, 0, 0, 0); }
ED_DEV long to_fp8x8(const uint4& u) {
  float f[8];
  unpack8(u, f);
  int lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  int hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], 0, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  return (long)(((unsigned long)(unsigned)hi << 32) | (unsigned)lo);
}
// k-step kc (32 head-dim elements) of row `row` of a bf16 row-major tile with pitch ld
template <int DH>
ED_DEV long frag8(const bf16_t* t, int ld, int row, int kc, int g) {
  const int d0 = kc * 32 + 8 * g;
  if (d0 >= DH) return 0;
  return to_fp8x8(*(const uint4*)(t + row * ld + d0));
}

// Stage one tensor (rows [S][DH] of head h of image b, row stride ld) for the hpb heads
// bh0 .. bh0+hpb-1 of the workgroup into LDS row-major [SP][DP] per head (rm + hl * rm_hs),
// zero padding (ONES: column DH of every valid row is 1.0 -- the forward's V denominator row).
// Loads are issued U at a time before their LDS writes.
template <int DH, int DP, int U, bool ONES = false>
ED_DEV void stage_heads_u(const bf16_t* __restrict__ base, long ld, int S, int SP, int H, int bh0, int hpb,
                          bf16_t* rm, int rm_hs, int r0 = 0) {
  constexpr int CH = DP / 8;
  const int ph = SP * CH, total = hpb * ph;
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * U) {
    uint4 v[U];
    int hl[U], r[U], c8[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * 256;
      hl[u] = hpb == 1 ? 0 : e / ph;
      const int t = e - hl[u] * ph;
      r[u] = t / CH;
      c8[u] = (t - r[u] * CH) * 8;
      v[u] = (uint4){0u, 0u, 0u, 0u};
      if (e < total && r0 + r[u] < S && c8[u] < DH) {
        const int bh = bh0 + hl[u], b = bh / H, h = bh - b * H;
        v[u] = *(const uint4*)(base + ((long)b * S + r0 + r[u]) * ld + h * DH + c8[u]);
      }
      if (ONES && e < total && r0 + r[u] < S && c8[u] == DH) v[u].x = 0x3F80u;  // bf16 1.0 in column DH
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (e0 + u * 256 >= total) break;
      *(uint4*)(rm + hl[u] * rm_hs + r[u] * DP + c8[u]) = v[u];
    }
  }
}
template <int DH, int DP, bool ONES = false>
ED_DEV void stage_heads(const bf16_t* __restrict__ base, long ld, int S, int SP, int H, int bh0, int hpb,
                        bf16_t* rm, int rm_hs, int r0 = 0) {
  // several heads (short sequences): 4 chunks per thread in flight; one long head: the
  // plain loop measured faster (fewer live registers in the 2-workgroup-per-CU kernels)
  if (hpb > 1) stage_heads_u<DH, DP, 4, ONES>(base, ld, S, SP, H, bh0, hpb, rm, rm_hs, r0);
  else stage_heads_u<DH, DP, 1, ONES>(base, ld, S, SP, H, bh0, hpb, rm, rm_hs, r0);
}

// K and V of the workgroup's heads in ONE pass (2*U loads per thread in flight): the forward's
// staging is one global round trip
template <int DH, int DP, int U, bool ONES>
ED_DEV void stage_kv_u(const bf16_t* __restrict__ kb, long ldk, const bf16_t* __restrict__ vb, long ldv, int S, int SP,
                       int H, int bh0, int hpb, bf16_t* ks, bf16_t* vs, int hs, int r0) {
  constexpr int CH = DP / 8;
  const int ph = SP * CH, total = hpb * ph;
  for (int e0 = threadIdx.x; e0 < total; e0 += 256 * U) {
    uint4 kv[U], vv[U];
    int off[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * 256;
      const int hl = hpb == 1 ? 0 : e / ph;
      const int t = e - hl * ph, r = t / CH, c8 = (t - r * CH) * 8;
      off[u] = hl * hs + r * DP + c8;
      kv[u] = (uint4){0u, 0u, 0u, 0u};
      vv[u] = kv[u];
      if (e < total && r0 + r < S && c8 < DH) {
        const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
        kv[u] = *(const uint4*)(kb + ((long)b * S + r0 + r) * ldk + h * DH + c8);
        vv[u] = *(const uint4*)(vb + ((long)b * S + r0 + r) * ldv + h * DH + c8);
      }
      if (ONES && e < total && r0 + r < S && c8 == DH) vv[u].x = 0x3F80u;  // bf16 1.0 in column DH
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (e0 + u * 256 >= total) break;
      *(uint4*)(ks + off[u]) = kv[u];
      *(uint4*)(vs + off[u]) = vv[u];
    }
  }
}

// Workgroup -> head-group index, XCD-aware: workgroup i runs on XCD i % 8, so consecutive head
// groups (the heads of one image share every 128-B row of the fused q / k / v projection) are
// given to consecutive workgroups OF ONE XCD and each row is fetched into one L2, not eight.
// Bijective when the grid is a multiple of 8 (else identity).
ED_DEV int xcd_group(int i, int n) { return (n & 7) ? i : (i & 7) * (n >> 3) + (i >> 3); }

// Cross-row reductions of the 4 lane rows (lane = 16 * g + l16) by the gfx950 permlane swaps
// (VALU, no LDS round trip as ds_bpermute): each returns the pair {v, v of lane ^ 16 / ^ 32}.
ED_DEV float max_x16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
ED_DEV float max_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
ED_DEV float sum_x16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
ED_DEV float sum_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

ED_DEV float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

#ifndef ED_ATTN_NT8
#define ED_ATTN_NT8 4  // dh 8 forward: 16-query tiles per wave task (A/B switch)
#endif
#ifndef ED_ATTN_FWD_UNROLL
#define ED_ATTN_FWD_UNROLL 2  // forward key loop unroll (32-key steps; A/B switch)
#endif
__host__ __device__ constexpr int fwd_tiles_per_task(int dh) { return dh == 8 ? ED_ATTN_NT8 : 2; }

template <bool B>
struct BoundTag {
  static constexpr bool value = B;
};
// Bound path of the forward: the log2-domain softmax offset of a query row is the Cauchy-Schwarz
// bound scale * log2e * |q| * max_k |k| (>= every score of the row), used only while it is <= this:
// the row's largest p is then >= 2^-2*FWD_BOUND_MAX (a normal fp32 / bf16 value), so the shifted
// exponentials are exact up to rounding and no running max, rescale or alpha exp is needed
constexpr float FWD_BOUND_MAX = 40.f;
ED_DEV float bf16_sq4(s4 v) {
  float a = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float f = __uint_as_float((unsigned)(unsigned short)v[i] << 16);
    a = __builtin_fmaf(f, f, a);
  }
  return a;
}

// Forward.  A wave task is a PAIR (dh 8: four) of 16-query tiles of one head: the K and V^T fragments
// read from LDS serve both, and the two online-softmax chains are independent.  Keys are
// consumed 32 at a time (two MFMA tiles) per softmax update; the running max is kept in the
// log2 domain (scale * log2 e) and p = exp2(s * scale * log2e - m) is one FMA + a raw
// v_exp_f32 (arguments <= 0, underflow to 0 is the correct limit).  MASK: key count not a
// multiple of 32 (keys past SK get -inf).  With every key of the head resident, a task whose
// rows have a small score bound (FWD_BOUND_MAX) uses that bound as a fixed offset instead of the
// running max (no max tree, no rescale of the accumulators): the same softmax up to rounding.
template <int DH, bool MASK, bool F8, int SC = 0>
__global__ __launch_bounds__(256) void attn_fwd_mfma(const EncdiffAttnArgs p, int hpb, int kch) {
  constexpr int DP = DH < 16 ? 16 : DH;
  constexpr int KC = DP / 16;
  constexpr bool ONES = DH == 8;   // denominator from the PV MFMA (V^T row 8 = 1)
  constexpr int KC8 = (DH + 31) / 32;  // fp8 score k-steps
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  // SC > 0: sq == sk == SC, one head per workgroup, K / V resident (compile-time loop bounds)
  const int H = p.heads, SQ = SC ? SC : p.sq, SK = SC ? SC : p.sk;
  if (SC) { hpb = 1; kch = (SC + 31) & ~31; }
  const int SKP = (SK + 31) & ~31;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int bh0 = xcd_group(blockIdx.x, gridDim.x) * hpb;
  const int KR = kch < SKP ? kch : SKP;  // key rows resident in LDS at a time
  bf16_t* Ks = sm;                        // [hpb][KR][DP]
  bf16_t* Vs = sm + hpb * KR * DP;        // [hpb][KR][DP], read transposed (ds_read_b64_tr_b16)
  float* kn = (float*)(sm + 2 * hpb * KR * DP);  // [hpb] max_k |k|^2 (resident K only)
  constexpr int NT = fwd_tiles_per_task(DH);  // 16-query tiles per wave task (independent chains)
  const int qtiles = (SQ + 15) >> 4, npairs = (qtiles + NT - 1) / NT;
  const float sl2 = p.scale * LOG2E;
  // per-task state: a pair of 16-query tiles of head hl
  int hl = 0, b = 0, h = 0, q[NT];
  s4 qf[NT][KC];
  long qf8[NT][KC8];
  float m[NT], l[NT];
  v4f o[NT][KC];
  auto init = [&](int task) {
    hl = task / npairs;
    const int qp = task - hl * npairs;
    const int bh = bh0 + hl;
    b = bh / H;
    h = bh - b * H;
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      q[u] = (NT * qp + u) * 16 + l16;
      const bool qv = q[u] < SQ;
      const bf16_t* qp_ = (const bf16_t*)p.q + ((long)b * SQ + q[u]) * p.ldq + h * DH;
      if constexpr (F8) {
#pragma unroll
        for (int kc = 0; kc < KC8; ++kc) {
          const int d0 = kc * 32 + 8 * g;
          qf8[u][kc] = (qv && d0 < DH) ? to_fp8x8(*(const uint4*)(qp_ + d0)) : 0;
        }
      } else {
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          const int d0 = kc * 16 + 4 * g;
          qf[u][kc] = (qv && d0 < DH) ? ld4(qp_ + d0) : (s4){0, 0, 0, 0};
        }
      }
      m[u] = -INFINITY;
      l[u] = 0.f;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) o[u][dt] = (v4f){0.f, 0.f, 0.f, 0.f};
    }
  };
  // bound path for the task's tiles (wave-uniform): m[u] = the rows' score bounds
  auto pick_bound = [&]() -> bool {
    if constexpr (F8 || DH > 32) {  // (dh 64 / 128: the second consume variant costs ~70 VGPRs)
      return false;
    } else {
      const float k2 = kn[hl];
      float mb[NT];
      bool ok = true;
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        float n2 = 0.f;
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) n2 += bf16_sq4(qf[u][kc]);
        n2 = sum_x32(sum_x16(n2));
        // small relative + absolute slack over the fp32 rounding of the MFMA dot products
        mb[u] = __builtin_amdgcn_sqrtf(n2 * k2) * sl2 * 1.001f + 1e-6f;  // raw v_sqrt (bound only)
        ok = ok && mb[u] <= FWD_BOUND_MAX;
      }
      if (!__all(ok)) return false;
#pragma unroll
      for (int u = 0; u < NT; ++u) m[u] = mb[u];
      return true;
    }
  };
  // keys [kbase, kbase + klen) of the task's head, staged at local rows 0 .. klen-1
  auto consume = [&](auto bnd, int kbase, int klen) {
    constexpr bool BOUND = decltype(bnd)::value;
    const bf16_t* kb = Ks + hl * KR * DP;
    const bf16_t* vb = Vs + hl * KR * DP;
#pragma unroll ED_ATTN_FWD_UNROLL
    for (int k0 = 0; k0 < klen; k0 += 32) {
      s4 kf[2][KC];
      long kf8[2][KC8];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if constexpr (F8) {
#pragma unroll
          for (int kc = 0; kc < KC8; ++kc) kf8[t][kc] = frag8<DH>(kb, DP, k0 + t * 16 + l16, kc, g);
        } else {
#pragma unroll
          for (int kc = 0; kc < KC; ++kc) kf[t][kc] = ld4(kb + (k0 + t * 16 + l16) * DP + kc * 16 + 4 * g);
        }
      }
      s4 pf[NT][2];
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        float sv[8];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          v4f sc = {0.f, 0.f, 0.f, 0.f};
          if constexpr (F8) {
#pragma unroll
            for (int kc = 0; kc < KC8; ++kc) sc = mma8(kf8[t][kc], qf8[u][kc], sc);
          } else {
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) sc = mma(kf[t][kc], qf[u][kc], sc);
          }
#pragma unroll
          for (int i = 0; i < 4; ++i)
            sv[4 * t + i] = (!MASK || kbase + k0 + t * 16 + 4 * g + i < SK) ? sc[i] : -INFINITY;
        }
        float mn = m[u], alpha = 1.f;
        if constexpr (!BOUND) {
          // max over raw scores (the scale is positive), the log2-domain max = that * sl2
          float tmax = fmaxf(fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3])),
                             fmaxf(fmaxf(sv[4], sv[5]), fmaxf(sv[6], sv[7])));
          tmax = max_x32(max_x16(tmax));
          mn = fmaxf(m[u], tmax * sl2);
          alpha = ex2(m[u] - mn);
          m[u] = mn;
        }
        float pv[8];
        {  // the exp arguments as packed pairs (v_pk_fma_f32: half the issue slots of 8 v_fma_f32)
          const v2f s2 = {sl2, sl2}, nm = {-mn, -mn};
#pragma unroll
          for (int i = 0; i < 8; i += 2) {
            const v2f a = __builtin_elementwise_fma((v2f){sv[i], sv[i + 1]}, s2, nm);
            pv[i] = ex2(a[0]);
            pv[i + 1] = ex2(a[1]);
          }
        }
        if constexpr (!ONES) {
          float ls = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) ls += pv[i];
          l[u] = BOUND ? l[u] + ls : l[u] * alpha + ls;
        }
        if constexpr (!BOUND) {
#pragma unroll
          for (int dt = 0; dt < KC; ++dt) o[u][dt] *= alpha;
        }
        pf[u][0] = pack4(pv[0], pv[1], pv[2], pv[3]);
        pf[u][1] = pack4(pv[4], pv[5], pv[6], pv[7]);
      }
#pragma unroll
      for (int dt = 0; dt < KC; ++dt)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const s4 vf = ldtr(vb, DP, k0 + t * 16, dt * 16, l16, g);  // V^T fragment
#pragma unroll
          for (int u = 0; u < NT; ++u) o[u][dt] = mma(vf, pf[u][t], o[u][dt]);
        }
    }
  };
  auto finish = [&]() {
#pragma unroll
    for (int u = 0; u < NT; ++u) {
      float lu;
      if constexpr (ONES) {
        // O^T row 8 (= g 2, register 0) is sum_k p for query l16: broadcast from lane 32 + l16
        lu = __shfl(o[u][0][0], 32 + l16, 64);
      } else {
        lu = l[u];
        lu = sum_x32(sum_x16(lu));
      }
      const float inv = __builtin_amdgcn_rcpf(lu);  // v_rcp_f32 (1 ulp; lu >= 1 or a normal bound-path sum)
      if (q[u] < SQ) {
        bf16_t* op = (bf16_t*)p.o + ((long)b * SQ + q[u]) * p.ldo + h * DH;
#pragma unroll
        for (int dt = 0; dt < KC; ++dt) {
          const int d0 = dt * 16 + 4 * g;
          if (d0 < DH) {
            uint2 w;
            w.x = pack2(o[u][dt][0] * inv, o[u][dt][1] * inv);
            w.y = pack2(o[u][dt][2] * inv, o[u][dt][3] * inv);
            *(uint2*)(op + d0) = w;
          }
        }
        if (g == 0 && p.lse) p.lse[(long)(bh0 + hl) * SQ + q[u]] = (m[u] + __log2f(lu)) * LN2;  // natural-log LSE
      }
    }
  };
  if (KR == SKP) {  // every head's K / V resident: waves loop over their tasks
    // (tasks split over blockIdx.y when the host spread a small grid over query blocks: workgroup
    // y takes tasks y, y + nqb, ...)
    const int ty = blockIdx.y, tny = gridDim.y, t0 = ty + tny * wave;
    // the first task's Q loads are issued with the K / V staging loads (one round trip)
    if (t0 < hpb * npairs) init(t0);
    if (tid < hpb) kn[tid] = 0.f;
    stage_kv_u<DH, DP, 2, ONES>((const bf16_t*)p.k, p.ldk, (const bf16_t*)p.v, p.ldv, SK, SKP, H, bh0, hpb, Ks, Vs,
                                SKP * DP, 0);
    __syncthreads();
    if constexpr (!F8 && DH <= 32) {  // max_k |k|^2 per head (LDS max over non-negative floats as ints)
      for (int r = tid; r < hpb * SKP; r += 256) {
        const int hr = r / SKP;
        const bf16_t* kr = Ks + hr * SKP * DP + (r - hr * SKP) * DP;
        float n2 = 0.f;
#pragma unroll
        for (int c = 0; c < DH; c += 4) n2 += bf16_sq4(*(const s4*)(kr + c));
        atomicMax((int*)&kn[hr], __float_as_int(n2));
      }
      __syncthreads();
    }
    for (int task = t0; task < hpb * npairs; task += 4 * tny) {
      if (task != t0) init(task);
      if constexpr (F8 || DH > 32) {
        consume(BoundTag<false>{}, 0, SKP);
      } else {
        if (pick_bound()) consume(BoundTag<true>{}, 0, SKP);
        else consume(BoundTag<false>{}, 0, SKP);
      }
      finish();
    }
    return;
  }
  // K / V longer than the LDS budget (one head per workgroup, hpb == 1): blockIdx.y picks four
  // query-tile pairs, one per wave, whose online softmax runs over key chunks of KR rows
  // streamed through LDS (every wave reaches every barrier)
  const int task = blockIdx.y * 4 + wave;
  const bool active = task < npairs;
  init(active ? task : 0);
  for (int c0 = 0; c0 < SKP; c0 += KR) {
    const int klen = SKP - c0 < KR ? SKP - c0 : KR;
    __syncthreads();  // the previous chunk is consumed
    stage_heads<DH, DP>((const bf16_t*)p.k, p.ldk, SK, klen, H, bh0, 1, Ks, KR * DP, c0);
    stage_heads<DH, DP, ONES>((const bf16_t*)p.v, p.ldv, SK, klen, H, bh0, 1, Vs, KR * DP, c0);
    __syncthreads();
    if (active) consume(BoundTag<false>{}, c0, klen);
  }
  if (active) finish();
}

// q-split of phase A: enough (key tile, query slice) tasks for the 4 waves
__device__ __host__ inline int attn_qsplit(int ktiles, int hpb) {
  const int t = ktiles * hpb;
  return t >= 4 ? 1 : (t >= 2 ? 2 : 4);
}

// dS^T row pitch in LDS: +16 elements (32 B) per row so the transposed reads of 8 consecutive
// rows fall on different banks
__device__ __host__ inline int ds_pitch(int sqp) { return sqp + 16; }
// The chunked dS^T (dsl > 1, S = 256) is instead unpadded with its 8-byte chunks XOR-swizzled per
// row: chunk c of row r sits at c ^ dsw(r & 15).  dsw was searched so that both the b64 stores (16
// rows x 2 chunks per half-wave) and the transposed b64 reads (4 rows x 4 chunks x 2 lane groups)
// hit 32 distinct bank pairs (the padded pitch left 2-way conflicts on the stores)
ED_DEV int dsw(int r) { return ((4 * r) ^ (2 * (r >> 3))) & 63; }
ED_DEV s4 ldtr_sw(const bf16_t* t, int ld, int r0, int c0, int l16, int g) {
  const int r = r0 + 4 * g + (l16 >> 2);
  const int c = ((c0 >> 2) + (l16 & 3)) ^ dsw(r & 15);
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(t + r * ld + 4 * c));
}

// split: phase A (dK, dV) and phase B (dQ, scores recomputed) run in two workgroups of their own
// (twice the workgroups per CU to hide each wave's LDS -> MFMA -> exp chains); both stage the
// head group.  The pair and consecutive head groups stay on one XCD (workgroup i runs on XCD i % 8).
template <int DH, bool MASK, bool F8, int SC = 0>
__global__ __launch_bounds__(256) void attn_bwd_mfma(const EncdiffAttnArgs p, int hpb, int dsl, int split) {
  constexpr int DP = DH < 16 ? 16 : DH;   // MFMA k extent of the head dim
  constexpr int RP = DH < 16 ? 8 : DH;    // LDS row pitch (dh = 8 staged unpadded)
  constexpr int KC = DP / 16;
  constexpr int KC8 = (DH + 31) / 32;
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  // SC > 0: sq == sk == SC and one head per workgroup known at compile time
  const int H = p.heads, SQ = SC ? SC : p.sq, SK = SC ? SC : p.sk;
  if (SC) hpb = 1;
  const int SQP = (SQ + 15) & ~15, SKP = (SK + 15) & ~15;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  int grp = blockIdx.x, part = -1;  // part: -1 both phases, 0 phase A only, 1 phase B only
  if (split) {
    const int n = gridDim.x;
    if (n & 15) {
      grp = blockIdx.x >> 1;
      part = blockIdx.x & 1;
    } else {
      const int s = blockIdx.x >> 3;
      grp = (blockIdx.x & 7) * (n >> 4) + (s >> 1);
      part = s & 1;
    }
  } else {
    grp = xcd_group(blockIdx.x, gridDim.x);
  }
  const int bh0 = grp * hpb;
  // per head, row-major: Q, dO [SQP][RP]; K, V [SKP][RP]; lse2, D [SQP]; (dsl) dS^T [SKP][SQP+16].
  // The transposed operands (Q^T, dO^T, K^T, dS^T) are read with ds_read_b64_tr_b16.
  const int QE = SQP * RP, KE = SKP * RP;
  const int oG = QE, oK = 2 * QE, oV = oK + KE;
  const int per_head = oV + KE;
  float* fls = (float*)(sm + hpb * per_head);
  const bool swz = dsl > 1 && (SQP & 255) == 0;  // swizzled chunked dS^T (dsw)
  const int DSP = swz ? SQP : ds_pitch(SQP);
  bf16_t* dS = (bf16_t*)(fls + hpb * 2 * SQP);  // [hpb][SKP][DSP] when dsl
  const int qtiles = SQP >> 4, ktiles = SKP >> 4;
  const int QS = attn_qsplit(ktiles, hpb);
  float* red = (float*)(dS + (dsl ? hpb * SKP * DSP : 0));  // phase-A partials [task][2][16*DP] when QS > 1
  // ONE staging pass, every load of a thread's chunk in flight together: Q, dO, O (query rows),
  // K, V (key rows), lse; D = rowsum(dO * O) summed over the row's CH chunk lanes by xor-shuffles
  {
    constexpr int CH = RP / 8;
    const int nq = hpb * SQP * CH, nk = hpb * SKP * CH, n = nq > nk ? nq : nk;
    for (int e0 = 0; e0 < n; e0 += 256) {
      const int e = e0 + tid;
      const uint4 z = {0u, 0u, 0u, 0u};
      uint4 qv = z, gv = z, ov = z, kv = z, vv = z;
      float lq = 0.f;
      const int hq = e / (SQP * CH), tq = e - hq * SQP * CH, rq = tq / CH, cq = (tq - rq * CH) * 8;
      const int hk = e / (SKP * CH), tk = e - hk * SKP * CH, rk = tk / CH, ck = (tk - rk * CH) * 8;
      if (e < nq && rq < SQ && cq < DH) {
        const int bh = bh0 + hq, b = bh / H, h = bh - b * H;
        const long row = (long)b * SQ + rq;
        qv = *(const uint4*)((const bf16_t*)p.q + row * p.ldq + h * DH + cq);
        gv = *(const uint4*)((const bf16_t*)p.d_o + row * p.lddo + h * DH + cq);
        ov = *(const uint4*)((const bf16_t*)p.o + row * p.ldo + h * DH + cq);
        lq = p.lse[(long)bh * SQ + rq] * LOG2E;
      }
      if (e < nk && rk < SK && ck < DH) {
        const int bh = bh0 + hk, b = bh / H, h = bh - b * H;
        const long row = (long)b * SK + rk;
        kv = *(const uint4*)((const bf16_t*)p.k + row * p.ldk + h * DH + ck);
        vv = *(const uint4*)((const bf16_t*)p.v + row * p.ldv + h * DH + ck);
      }
      float a[8], c[8], d = 0.f;
      unpack8(ov, a);
      unpack8(gv, c);
#pragma unroll
      for (int k = 0; k < 8; ++k) d += a[k] * c[k];
#pragma unroll
      for (int s = 1; s < CH; s <<= 1) d += __shfl_xor(d, s, 64);
      if (e < nq) {
        bf16_t* hb = sm + hq * per_head + rq * RP + cq;
        *(uint4*)hb = qv;
        *(uint4*)(hb + oG) = gv;
        if (cq == 0) {
          // both row constants stored NEGATED: -lse2 is the exp argument's addend and -D the dP
          // accumulator's initial value (no sign flips in the per-score loops)
          fls[hq * 2 * SQP + rq] = -lq;
          fls[hq * 2 * SQP + SQP + rq] = -d;
        }
      }
      if (e < nk) {
        bf16_t* hb = sm + hk * per_head + rk * RP + ck;
        *(uint4*)(hb + oK) = kv;
        *(uint4*)(hb + oV) = vv;
      }
    }
  }
  __syncthreads();
  const float scale = p.scale, sl2 = p.scale * LOG2E;
  // row fragment (A or B operand with k = head dim) of a row-major staged tile
  auto rowf = [&](const bf16_t* t, int row, int kc) -> s4 {
    // dh 8 (unpadded rows): lanes g >= 2 hold the zero k = 8..15 half of the fragment; their load
    // stays inside the row and is discarded by a select (no exec-mask branch)
    const s4 v = ld4(t + row * RP + kc * 16 + 4 * (DH < 16 ? (g & 1) : g));
    return (DH < 16 && g >= 2) ? (s4){0, 0, 0, 0} : v;
  };
  // the same fragment WITHOUT zeroing the k = 8..15 half (dh = 8: lanes g >= 2 hold a duplicate of
  // the row's k = 0..7, finite values): for the operand of an MFMA whose other operand was built by
  // rowf -- its zero half cancels them -- so the per-query-tile loops issue no selects
  auto rowf_raw = [&](const bf16_t* t, int row, int kc) -> s4 {
    return ld4(t + row * RP + kc * 16 + 4 * (DH < 16 ? (g & 1) : g));
  };
  if (dsl > 1) {
    // Key chunks of dsl keys (one head, host-checked: hpb 1, <= 16 query tiles): phase A on the
    // chunk's key tiles leaves the chunk's dS^T in LDS, phase B adds the chunk's share of dQ^T
    // into registers kept across chunks (each wave owns query tiles wave, wave + 4, ...).  No
    // score is computed twice, and the small dS^T buffer keeps three workgroups per CU.
    const int KCH = dsl;
    const bf16_t *Qs = sm, *Gs = sm + oG, *Ks = sm + oK, *Vs = sm + oV;
    const float* lse = fls;
    const float* Dv = fls + SQP;
    const int b = bh0 / H, h = bh0 - b * H;
    v4f dq[4][KC];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) dq[j][dt] = (v4f){0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < SKP; c0 += KCH) {
      const int nkt = (SKP - c0 < KCH ? SKP - c0 : KCH) >> 4;
      for (int t = wave; t < nkt; t += 4) {
        const int key = c0 + t * 16 + l16;
        const bool kv = key < SK;
        s4 kf[KC], vf[KC];
        long kf8[KC8];
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          kf[kc] = rowf(Ks, key, kc);
          vf[kc] = rowf(Vs, key, kc);
        }
        if constexpr (F8) {
#pragma unroll
          for (int kc = 0; kc < KC8; ++kc) kf8[kc] = frag8<DH>(Ks, RP, key, kc, g);
        }
        v4f dk[2][KC], dv[2][KC];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int dt = 0; dt < KC; ++dt) { dk[u][dt] = (v4f){0.f, 0.f, 0.f, 0.f}; dv[u][dt] = dk[u][dt]; }
        auto qstep = [&](const int qt, const int u) {
          // dP starts from -D (the row constant in the accumulator): dS = P * dP needs no subtraction
          const float4 dv4 = *(const float4*)(Dv + qt * 16 + 4 * g);
          v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {dv4.x, dv4.y, dv4.z, dv4.w};
          if constexpr (F8) {
#pragma unroll
            for (int kc = 0; kc < KC8; ++kc) s = mma8(frag8<DH>(Qs, RP, qt * 16 + l16, kc, g), kf8[kc], s);
          }
#pragma unroll
          for (int kc = 0; kc < KC; ++kc) {
            if constexpr (!F8) s = mma(rowf_raw(Qs, qt * 16 + l16, kc), kf[kc], s);
            dp = mma(rowf_raw(Gs, qt * 16 + l16, kc), vf[kc], dp);
          }
          float pv[4], ds[4];
          {  // exp arguments as packed pairs (v_pk_fma_f32)
            const int q0 = qt * 16 + 4 * g;
            const v2f sl = {sl2, sl2};
#pragma unroll
            for (int i = 0; i < 4; i += 2) {
              const v2f e = __builtin_elementwise_fma((v2f){s[i], s[i + 1]}, sl, (v2f){lse[q0 + i], lse[q0 + i + 1]});
              pv[i] = (!MASK || (kv && q0 + i < SQ)) ? ex2(e[0]) : 0.f;
              pv[i + 1] = (!MASK || (kv && q0 + i + 1 < SQ)) ? ex2(e[1]) : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) ds[i] = pv[i] * dp[i];
          }
          const s4 pf = pack4(pv[0], pv[1], pv[2], pv[3]);
          const s4 df = pack4(ds[0], ds[1], ds[2], ds[3]);
          *(s4*)(dS + (t * 16 + l16) * DSP + 4 * (swz ? (qt * 4 + g) ^ dsw(l16) : qt * 4 + g)) = df;
#pragma unroll
          for (int dt = 0; dt < KC; ++dt) {
            dv[u][dt] = mma(ldtr(Gs, RP, qt * 16, dt * 16, l16, g), pf, dv[u][dt]);
            dk[u][dt] = mma(ldtr(Qs, RP, qt * 16, dt * 16, l16, g), df, dk[u][dt]);
          }
        };
        int qt0 = 0;
#pragma unroll 4
        for (; qt0 + 1 < qtiles; qt0 += 2) {
          qstep(qt0, 0);
          qstep(qt0 + 1, 1);
        }
        if (qt0 < qtiles) qstep(qt0, 0);
        if (kv) {
          bf16_t* dkp = (bf16_t*)p.dk + ((long)b * SK + key) * p.lddk + h * DH;
          bf16_t* dvp = (bf16_t*)p.dv + ((long)b * SK + key) * p.lddv + h * DH;
#pragma unroll
          for (int dt = 0; dt < KC; ++dt) {
            const int d0 = dt * 16 + 4 * g;
            if (d0 < DH) {
              const v4f a = dk[0][dt] + dk[1][dt], c = dv[0][dt] + dv[1][dt];
              uint2 w;
              w.x = pack2(a[0] * scale, a[1] * scale);
              w.y = pack2(a[2] * scale, a[3] * scale);
              *(uint2*)(dkp + d0) = w;
              w.x = pack2(c[0], c[1]);
              w.y = pack2(c[2], c[3]);
              *(uint2*)(dvp + d0) = w;
            }
          }
        }
      }
      __syncthreads();  // the chunk's dS^T is complete
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int qt = wave + 4 * j;
        if (qt < qtiles) {
          for (int t = 0; t < nkt; ++t) {
            const s4 df = swz ? ldtr_sw(dS, DSP, t * 16, qt * 16, l16, g) : ldtr(dS, DSP, t * 16, qt * 16, l16, g);
#pragma unroll
            for (int dt = 0; dt < KC; ++dt) dq[j][dt] = mma(ldtr(Ks, RP, c0 + t * 16, dt * 16, l16, g), df, dq[j][dt]);
          }
        }
      }
      __syncthreads();  // dS^T is rewritten by the next chunk
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = (wave + 4 * j) * 16 + l16;
      if (wave + 4 * j < qtiles && q < SQ) {
        bf16_t* dqp = (bf16_t*)p.dq + ((long)b * SQ + q) * p.lddq + h * DH;
#pragma unroll
        for (int dt = 0; dt < KC; ++dt) {
          const int d0 = dt * 16 + 4 * g;
          if (d0 < DH) {
            uint2 w;
            w.x = pack2(dq[j][dt][0] * scale, dq[j][dt][1] * scale);
            w.y = pack2(dq[j][dt][2] * scale, dq[j][dt][3] * scale);
            *(uint2*)(dqp + d0) = w;
          }
        }
      }
    }
    return;
  }
  // ---- phase A: dK, dV (task = key tile x query slice; query tiles in pairs) ----------
  const int ntA = part == 1 ? 0 : hpb * ktiles * QS;
  for (int task = wave; task < ntA; task += 4) {
    const int hl = task / (ktiles * QS), rem = task - hl * ktiles * QS;
    const int kt = rem / QS, qs = rem - kt * QS;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    const bf16_t* base = sm + hl * per_head;
    const bf16_t *Qs = base, *Gs = base + oG;
    const bf16_t *Ks = base + oK, *Vs = base + oV;
    const float* lse = fls + hl * 2 * SQP;
    const float* Dv = lse + SQP;
    bf16_t* dSh = dS + hl * SKP * DSP;
    const int key = kt * 16 + l16;
    const bool kv = key < SK;
    s4 kf[KC], vf[KC];
    long kf8[KC8];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      kf[kc] = rowf(Ks, key, kc);
      vf[kc] = rowf(Vs, key, kc);
    }
    if constexpr (F8) {
#pragma unroll
      for (int kc = 0; kc < KC8; ++kc) kf8[kc] = frag8<DH>(Ks, RP, key, kc, g);
    }
    v4f dk[2][KC], dv[2][KC];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) { dk[u][dt] = (v4f){0.f, 0.f, 0.f, 0.f}; dv[u][dt] = dk[u][dt]; }
    // the two query tiles of a step are independent chains (LDS read -> MFMA -> exp -> MFMA);
    // without a partial last step they are straight-line code the compiler interleaves
    auto qstep = [&](const int qt, const int u) {
        // dP starts from -D (the row constant in the accumulator): dS = P * dP needs no subtraction
        const float4 dv4 = *(const float4*)(Dv + qt * 16 + 4 * g);
        v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {dv4.x, dv4.y, dv4.z, dv4.w};
        if constexpr (F8) {
#pragma unroll
          for (int kc = 0; kc < KC8; ++kc) s = mma8(frag8<DH>(Qs, RP, qt * 16 + l16, kc, g), kf8[kc], s);
        }
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          if constexpr (!F8) s = mma(rowf_raw(Qs, qt * 16 + l16, kc), kf[kc], s);
          dp = mma(rowf_raw(Gs, qt * 16 + l16, kc), vf[kc], dp);
        }
        float pv[4], ds[4];
        {  // exp arguments as packed pairs (v_pk_fma_f32)
          const int q0 = qt * 16 + 4 * g;
          const v2f sl = {sl2, sl2};
#pragma unroll
          for (int i = 0; i < 4; i += 2) {
            const v2f e = __builtin_elementwise_fma((v2f){s[i], s[i + 1]}, sl, (v2f){lse[q0 + i], lse[q0 + i + 1]});
            pv[i] = (!MASK || (kv && q0 + i < SQ)) ? ex2(e[0]) : 0.f;
            pv[i + 1] = (!MASK || (kv && q0 + i + 1 < SQ)) ? ex2(e[1]) : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 4; ++i) ds[i] = pv[i] * dp[i];
        }
        const s4 pf = pack4(pv[0], pv[1], pv[2], pv[3]);
        const s4 df = pack4(ds[0], ds[1], ds[2], ds[3]);
        if (dsl) *(s4*)(dSh + key * DSP + qt * 16 + 4 * g) = df;  // dS^T[key][q .. q+3] for phase B
#pragma unroll
        for (int dt = 0; dt < KC; ++dt) {
          dv[u][dt] = mma(ldtr(Gs, RP, qt * 16, dt * 16, l16, g), pf, dv[u][dt]);  // dO^T fragment
          dk[u][dt] = mma(ldtr(Qs, RP, qt * 16, dt * 16, l16, g), df, dk[u][dt]);  // Q^T fragment
        }
    };
    if (qtiles % (2 * QS) == 0) {
#pragma unroll
      for (int qt0 = qs; qt0 < qtiles; qt0 += 2 * QS) {
        qstep(qt0, 0);
        qstep(qt0 + QS, 1);
      }
    } else {
      for (int qt0 = qs; qt0 < qtiles; qt0 += 2 * QS) {
        qstep(qt0, 0);
        if (qt0 + QS < qtiles) qstep(qt0 + QS, 1);
      }
    }
#pragma unroll
    for (int dt = 0; dt < KC; ++dt) { dk[0][dt] += dk[1][dt]; dv[0][dt] += dv[1][dt]; }
    if (QS > 1) {  // partials of this query slice -> LDS, summed in slice order below
      float* r = red + (long)task * 2 * 16 * DP;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          r[(dt * 4 + i) * 64 + lane] = dk[0][dt][i];
          r[16 * DP + (dt * 4 + i) * 64 + lane] = dv[0][dt][i];
        }
    } else if (kv) {
      bf16_t* dkp = (bf16_t*)p.dk + ((long)b * SK + key) * p.lddk + h * DH;
      bf16_t* dvp = (bf16_t*)p.dv + ((long)b * SK + key) * p.lddv + h * DH;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < DH) {
          uint2 w;
          w.x = pack2(dk[0][dt][0] * scale, dk[0][dt][1] * scale);
          w.y = pack2(dk[0][dt][2] * scale, dk[0][dt][3] * scale);
          *(uint2*)(dkp + d0) = w;
          w.x = pack2(dv[0][dt][0], dv[0][dt][1]);
          w.y = pack2(dv[0][dt][2], dv[0][dt][3]);
          *(uint2*)(dvp + d0) = w;
        }
      }
    }
  }
  if (QS > 1 || dsl) __syncthreads();
  if (QS > 1 && part != 1) {
    // one wave per (head, key tile) adds its QS slices in order and writes dK, dV
    for (int t = wave; t < hpb * ktiles; t += 4) {
      const int hl = t / ktiles, kt = t - hl * ktiles;
      const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
      const int key = kt * 16 + l16;
      const float* r0 = red + (long)(t * QS) * 2 * 16 * DP;
      if (key < SK) {
        bf16_t* dkp = (bf16_t*)p.dk + ((long)b * SK + key) * p.lddk + h * DH;
        bf16_t* dvp = (bf16_t*)p.dv + ((long)b * SK + key) * p.lddv + h * DH;
#pragma unroll
        for (int dt = 0; dt < KC; ++dt) {
          const int d0 = dt * 16 + 4 * g;
          if (d0 >= DH) continue;
          float a[4], c[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            a[i] = 0.f; c[i] = 0.f;
            for (int qs = 0; qs < QS; ++qs) {
              a[i] += r0[(long)qs * 2 * 16 * DP + (dt * 4 + i) * 64 + lane];
              c[i] += r0[(long)qs * 2 * 16 * DP + 16 * DP + (dt * 4 + i) * 64 + lane];
            }
          }
          uint2 w;
          w.x = pack2(a[0] * scale, a[1] * scale);
          w.y = pack2(a[2] * scale, a[3] * scale);
          *(uint2*)(dkp + d0) = w;
          w.x = pack2(c[0], c[1]);
          w.y = pack2(c[2], c[3]);
          *(uint2*)(dvp + d0) = w;
        }
      }
    }
  }
  // ---- phase B: dQ (waves own query tiles; key tiles in pairs) ----------------------
  for (int task = wave; task < (part == 0 ? 0 : hpb * qtiles); task += 4) {
    const int hl = task / qtiles, qt = task - hl * qtiles;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    const bf16_t* base = sm + hl * per_head;
    const bf16_t *Qs = base, *Gs = base + oG;
    const bf16_t *Ks = base + oK, *Vs = base + oV;
    const float* lse = fls + hl * 2 * SQP;
    const float* Dv = lse + SQP;
    const bf16_t* dSh = dS + hl * SKP * DSP;
    const int q = qt * 16 + l16;
    const bool qv = q < SQ;
    v4f dq[2][KC];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) dq[u][dt] = (v4f){0.f, 0.f, 0.f, 0.f};
    if (dsl) {  // dS^T from phase A: MFMAs only
      auto kstep = [&](const int kt, const int u) {
        const s4 df = ldtr(dSh, DSP, kt * 16, qt * 16, l16, g);  // dS^T[key 4g+i][query l16]
#pragma unroll
        for (int dt = 0; dt < KC; ++dt)
          dq[u][dt] = mma(ldtr(Ks, RP, kt * 16, dt * 16, l16, g), df, dq[u][dt]);  // K^T fragment
      };
      int kt0 = 0;
#pragma unroll
      for (; kt0 + 1 < ktiles; kt0 += 2) {
        kstep(kt0, 0);
        kstep(kt0 + 1, 1);
      }
      if (kt0 < ktiles) kstep(kt0, 0);
    } else {
      const float nlq = lse[q], nDq = Dv[q];  // -lse2, -D (stored negated)
      s4 qf[KC], gf[KC];
      long qf8[KC8];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        qf[kc] = rowf(Qs, q, kc);
        gf[kc] = rowf(Gs, q, kc);
      }
      if constexpr (F8) {
#pragma unroll
        for (int kc = 0; kc < KC8; ++kc) qf8[kc] = frag8<DH>(Qs, RP, q, kc, g);
      }
      auto kstep = [&](const int kt, const int u) {
        v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {nDq, nDq, nDq, nDq};  // dP^T - D from the accumulator
        if constexpr (F8) {
#pragma unroll
          for (int kc = 0; kc < KC8; ++kc) st = mma8(frag8<DH>(Ks, RP, kt * 16 + l16, kc, g), qf8[kc], st);
        }
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          if constexpr (!F8) st = mma(rowf_raw(Ks, kt * 16 + l16, kc), qf[kc], st);
          dpt = mma(rowf_raw(Vs, kt * 16 + l16, kc), gf[kc], dpt);
        }
        float ds[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key = kt * 16 + 4 * g + i;
          const float pr = (!MASK || (qv && key < SK)) ? ex2(__builtin_fmaf(st[i], sl2, nlq)) : 0.f;
          ds[i] = pr * dpt[i];
        }
        const s4 df = pack4(ds[0], ds[1], ds[2], ds[3]);
#pragma unroll
        for (int dt = 0; dt < KC; ++dt)
          dq[u][dt] = mma(ldtr(Ks, RP, kt * 16, dt * 16, l16, g), df, dq[u][dt]);  // K^T fragment
      };
      int kt0 = 0;
#pragma unroll
      for (; kt0 + 1 < ktiles; kt0 += 2) {
        kstep(kt0, 0);
        kstep(kt0 + 1, 1);
      }
      if (kt0 < ktiles) kstep(kt0, 0);
    }
    if (qv) {
      bf16_t* dqp = (bf16_t*)p.dq + ((long)b * SQ + q) * p.lddq + h * DH;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < DH) {
          const v4f t = dq[0][dt] + dq[1][dt];
          uint2 w;
          w.x = pack2(t[0] * scale, t[1] * scale);
          w.y = pack2(t[2] * scale, t[3] * scale);
          *(uint2*)(dqp + d0) = w;
        }
      }
    }
  }
}

int mfma_hpb(const EncdiffAttnArgs& a) {
  int hpb = a.sq >= 64 ? 1 : 4;
  while (hpb > 1 && a.heads % hpb) hpb >>= 1;
  return hpb;
}

#ifndef ATTN_FWD_QSPLIT
#define ATTN_FWD_QSPLIT 1
#endif
template <int DH, bool F8>
int launch_mfma_fwd(const EncdiffAttnArgs& a, hipStream_t s) {
  constexpr int DP = DH < 16 ? 16 : DH;
  int hpb = mfma_hpb(a);
  const int SKP = (a.sk + 31) & ~31;
  size_t lds = (size_t)hpb * 2 * SKP * DP * sizeof(bf16_t) + 16 * sizeof(float);  // + the key norms
  int kch = SKP, nqb = 1;
  if (lds > 160 * 1024) {
    // K / V of a head exceed LDS (the VQ AttnBlock at 32x32 = 1024 tokens, dh 128): one head per
    // workgroup, key chunks of <= 64 KB streamed, query tiles split over blockIdx.y
    hpb = 1;
    kch = (int)((64 * 1024) / (2 * DP * sizeof(bf16_t))) & ~31;
    if (kch < 32) return ENCDIFF_ERR_SHAPE;
    constexpr int NT = fwd_tiles_per_task(DH);
    const int npairs = (((a.sq + 15) >> 4) + NT - 1) / NT;
    nqb = (npairs + 3) / 4;
    lds = (size_t)2 * kch * DP * sizeof(bf16_t);
  }
  // wide single-head blocks with few (image, head) workgroups (the VQ AttnBlock at 16x16: 128
  // workgroups of 128 KB K / V): query tasks spread over blockIdx.y, each workgroup staging the
  // head's K / V, so every CU takes one (up to 4 tasks per workgroup, one per wave)
  if (nqb == 1 && DH >= 64 && hpb == 1 && ATTN_FWD_QSPLIT) {
    constexpr int NT = fwd_tiles_per_task(DH);
    const int npairs = (((a.sq + 15) >> 4) + NT - 1) / NT;
    const int nx = a.batch * a.heads;
    while (nqb * 2 * nx <= 256 && npairs >= 4 * nqb * 2) nqb *= 2;
  }
  const dim3 grid(a.batch * a.heads / hpb, nqb);
  const bool mask = a.sk % 32 != 0;
  static const hipError_t attr0 = hipFuncSetAttribute((const void*)attn_fwd_mfma<DH, false, F8>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  static const hipError_t attr1 = hipFuncSetAttribute((const void*)attn_fwd_mfma<DH, true, F8>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr0; (void)attr1;
  if constexpr (DH == 8 && !F8) {
    if (a.sq == 256 && a.sk == 256 && hpb == 1 && nqb == 1) {  // level-0 self-attention of the UNet
      static const hipError_t attr2 = hipFuncSetAttribute((const void*)attn_fwd_mfma<DH, false, F8, 256>,
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)attr2;
      hipLaunchKernelGGL((attn_fwd_mfma<DH, false, F8, 256>), grid, dim3(256), lds, s, a, hpb, kch);
      ED_CHECK_LAUNCH();
      return ENCDIFF_OK;
    }
  }
  if (mask) hipLaunchKernelGGL((attn_fwd_mfma<DH, true, F8>), grid, dim3(256), lds, s, a, hpb, kch);
  else hipLaunchKernelGGL((attn_fwd_mfma<DH, false, F8>), grid, dim3(256), lds, s, a, hpb, kch);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

template <int DH, bool F8>
int launch_mfma_bwd(const EncdiffAttnArgs& a, hipStream_t s) {
  constexpr int DP = DH < 16 ? 16 : DH;
  constexpr int RP = DH < 16 ? 8 : DH;
  const int hpb = mfma_hpb(a);
  const int SQP = (a.sq + 15) & ~15, SKP = (a.sk + 15) & ~15;
  const int nblk = a.batch * a.heads / hpb;
  const int QS = attn_qsplit(SKP / 16, hpb);
  const size_t red = QS > 1 ? (size_t)hpb * (SKP / 16) * QS * 2 * 16 * DP * sizeof(float) : 0;
  const size_t base = (size_t)hpb * ((2 * SQP + 2 * SKP) * RP * sizeof(bf16_t) + 2 * SQP * sizeof(float)) + red;
  const size_t dsz = (size_t)hpb * SKP * ds_pitch(SQP) * sizeof(bf16_t);
  // dS^T kept in LDS for phase B (no second exp sweep) only while >= 3 workgroups fit a CU: at
  // one workgroup per CU (S = 256: 157 KB) every wave's LDS -> MFMA -> exp chain is exposed
  static const long dsl_max = [] {
    const char* e = getenv("ENCDIFF_ATTN_DSL_MAX");  // tuning knob (bytes)
    return e ? atol(e) : 52L * 1024;
  }();
  int dsl = (long)(base + dsz) <= dsl_max ? 1 : 0;
  size_t lds = base + (dsl ? dsz : 0);
  static const int kch_env = [] {
    const char* e = getenv("ENCDIFF_ATTN_KCHUNK");  // tuning knob (keys per dS^T chunk, 0: off)
    return e ? atoi(e) : 64;
  }();
  if (!dsl && kch_env >= 16 && hpb == 1 && QS == 1 && SQP <= 256 && SKP > kch_env) {
    const size_t csz = (size_t)kch_env * ds_pitch(SQP) * sizeof(bf16_t);
    if ((long)(base + csz) <= dsl_max + 4096) {
      dsl = kch_env & ~15;
      lds = base + csz;
    }
  }
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr0 = hipFuncSetAttribute((const void*)attn_bwd_mfma<DH, false, F8>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  static const hipError_t attr1 = hipFuncSetAttribute((const void*)attn_bwd_mfma<DH, true, F8>,
                                                      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr0; (void)attr1;
  // phase B recomputes the scores: optionally in workgroups of its own (measured: 59 -> 62 us at
  // S = 256 dh 8, B = 128 -- the workgroups already fill the CUs; kept as a knob)
  static const int split_env = [] {
    const char* e = getenv("ENCDIFF_ATTN_SPLIT");
    return e ? atoi(e) : 0;
  }();
  const int split = (dsl || !split_env) ? 0 : 1;  // (dsl > 1: chunked dS^T, one workgroup per head)
  const dim3 grid(nblk * (split ? 2 : 1));
  if constexpr (DH == 8 && !F8) {
    if (a.sq == 256 && a.sk == 256 && hpb == 1 && dsl != 1) {  // level-0 self-attention of the UNet
      static const hipError_t attr2 = hipFuncSetAttribute((const void*)attn_bwd_mfma<DH, false, F8, 256>,
                                                          hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      (void)attr2;
      hipLaunchKernelGGL((attn_bwd_mfma<DH, false, F8, 256>), grid, dim3(256), lds, s, a, hpb, dsl, split);
      ED_CHECK_LAUNCH();
      return ENCDIFF_OK;
    }
  }
  if (a.sq % 16 || a.sk % 16)
    hipLaunchKernelGGL((attn_bwd_mfma<DH, true, F8>), grid, dim3(256), lds, s, a, hpb, dsl, split);
  else hipLaunchKernelGGL((attn_bwd_mfma<DH, false, F8>), grid, dim3(256), lds, s, a, hpb, dsl, split);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

template <bool F8>
int dispatch_dh(const EncdiffAttnArgs& a, bool bwd, hipStream_t s) {
  switch (a.dh) {
    case 8: return bwd ? launch_mfma_bwd<8, F8>(a, s) : launch_mfma_fwd<8, F8>(a, s);
    case 16: return bwd ? launch_mfma_bwd<16, F8>(a, s) : launch_mfma_fwd<16, F8>(a, s);
    case 32: return bwd ? launch_mfma_bwd<32, F8>(a, s) : launch_mfma_fwd<32, F8>(a, s);
    // wider UNets (configs[4], model_channels=128: C=512 over 8 heads at the 8x8 / 4x4 levels)
    case 64: return bwd ? launch_mfma_bwd<64, F8>(a, s) : launch_mfma_fwd<64, F8>(a, s);
    default: return ENCDIFF_ERR_UNSUPPORTED;
  }
}

int attn_dispatch(const EncdiffAttnArgs* a, bool bwd, void* stream) {
  if (!a || !a->q || !a->k || !a->v || !a->o) return ENCDIFF_ERR_ARG;
  if (a->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_UNSUPPORTED;  // fp32: forward entry only
  if (bwd && (!a->d_o || !a->dq || !a->dk || !a->dv || !a->lse)) return ENCDIFF_ERR_ARG;
  if (a->batch <= 0 || a->heads <= 0 || a->sq <= 0 || a->sk <= 0 || a->dh % 8) return ENCDIFF_ERR_SHAPE;
  if (a->batch * a->heads % mfma_hpb(*a)) return ENCDIFF_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  if (a->dh == 128) {  // single-head AttnBlock of the VQ encoder (model.py AttnBlock): forward only (frozen)
    if (bwd || a->fp8_qk) return ENCDIFF_ERR_UNSUPPORTED;
    return launch_mfma_fwd<128, false>(*a, s);
  }
  return a->fp8_qk ? dispatch_dh<true>(*a, bwd, s) : dispatch_dh<false>(*a, bwd, s);
}

}  // namespace

extern "C" int encdiff_attention_fwd(const EncdiffAttnArgs* a, void* stream) {
  if (a && a->dtype == ENCDIFF_DT_F32) return ed_attention_fwd_f32(a, (hipStream_t)stream);
  if (a && a->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_ARG;
  return attn_dispatch(a, false, stream);
}
extern "C" int encdiff_attention_bwd(const EncdiffAttnArgs* a, void* stream) {
  if (a && a->dtype == ENCDIFF_DT_F32) return ed_attention_bwd_f32(a, (hipStream_t)stream);
  return attn_dispatch(a, true, stream);
}
