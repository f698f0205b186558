// attn_mfma.hip -- MFMA attention for the SpatialTransformer heads (attention.py:170-193).
//
// v_mfma_f32_16x16x16_bf16 (K = 16) tiles; head dims 8/16/32 are zero-padded to 16/16/32.
// Forward: per wave a 16-query tile; S^T = K Q^T is computed "swapped" so each lane holds
// 4 consecutive keys of ONE query: the row max / sum of the online softmax are in-register
// plus two cross-lane xor-shuffles, and the bf16 P is already the B operand of
// O^T = V^T P^T (no LDS round trip for P).  K and V^T of the block's heads live in LDS.
// Backward (recompute from LSE, no score matrix in HBM): phase A -- waves own key tiles and
// accumulate dK^T, dV^T over all query tiles; phase B -- waves own query tiles and
// accumulate dQ^T over all key tiles.  Q, K, V, dO and the transposed copies Q^T, K^T, dO^T
// are staged in LDS once per (image, head group); rowsum(dO * O) is computed while staging.
#include "common.h"

namespace {

typedef short s4 __attribute__((ext_vector_type(4)));

ED_DEV v4f mma(const s4& a, const s4& b, const v4f& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}
ED_DEV s4 ld4(const bf16_t* p) { return *(const s4*)p; }
ED_DEV s4 pack4(float a, float b, float c, float d) {
  s4 r;
  r[0] = (short)f2bf(a); r[1] = (short)f2bf(b); r[2] = (short)f2bf(c); r[3] = (short)f2bf(d);
  return r;
}

// stage rows [n][dh] of a head from a [rows][ld] tensor into LDS row-major [np][DP]
// (and optionally transposed [DP][np]); zero padding for rows >= n and dims >= dh.
template <int DH, int DP>
ED_DEV void stage_rows(const bf16_t* __restrict__ src, long ld, int n, int np, bf16_t* rm, bf16_t* tr, int tid,
                       int nthr) {
  constexpr int CH = DP / 8;  // 16-byte chunks per padded row
  for (int e = tid; e < np * CH; e += nthr) {
    const int r = e / CH, c8 = (e - r * CH) * 8;
    uint4 v = {0u, 0u, 0u, 0u};
    if (r < n && c8 < DH) v = *(const uint4*)(src + (long)r * ld + c8);
    *(uint4*)(rm + r * DP + c8) = v;
    if (tr) {
      const bf16_t* h = (const bf16_t*)&v;
#pragma unroll
      for (int k = 0; k < 8; ++k) tr[(c8 + k) * np + r] = h[k];
    }
  }
}

template <int DH>
__global__ __launch_bounds__(256) void attn_fwd_mfma(const EncdiffAttnArgs p, int hpb) {
  constexpr int DP = DH < 16 ? 16 : DH;
  constexpr int KC = DP / 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  const int H = p.heads, SQ = p.sq, SK = p.sk;
  const int SKP = (SK + 15) & ~15;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int bh0 = blockIdx.x * hpb;
  bf16_t* Ks = sm;                        // [hpb][SKP][DP]
  bf16_t* Vt = sm + hpb * SKP * DP;       // [hpb][DP][SKP]
  for (int hl = 0; hl < hpb; ++hl) {
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    stage_rows<DH, DP>((const bf16_t*)p.k + (long)b * SK * p.ldk + h * DH, p.ldk, SK, SKP, Ks + hl * SKP * DP,
                       nullptr, tid, 256);
    // V transposed only
    constexpr int CH = DP / 8;
    for (int e = tid; e < SKP * CH; e += 256) {
      const int r = e / CH, c8 = (e - r * CH) * 8;
      uint4 v = {0u, 0u, 0u, 0u};
      if (r < SK && c8 < DH) v = *(const uint4*)((const bf16_t*)p.v + ((long)b * SK + r) * p.ldv + h * DH + c8);
      const bf16_t* hv = (const bf16_t*)&v;
#pragma unroll
      for (int k = 0; k < 8; ++k) Vt[hl * DP * SKP + (c8 + k) * SKP + r] = hv[k];
    }
  }
  __syncthreads();
  const int qtiles = (SQ + 15) >> 4;
  const float scale = p.scale;
  for (int task = wave; task < hpb * qtiles; task += 4) {
    const int hl = task / qtiles, qt = task - hl * qtiles;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    const int q = qt * 16 + l16;
    const bool qv = q < SQ;
    const bf16_t* qp = (const bf16_t*)p.q + ((long)b * SQ + q) * p.ldq + h * DH;
    s4 qf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      const int d0 = kc * 16 + 4 * g;
      qf[kc] = (qv && d0 < DH) ? ld4(qp + d0) : (s4){0, 0, 0, 0};
    }
    const bf16_t* kb = Ks + hl * SKP * DP;
    const bf16_t* vb = Vt + hl * DP * SKP;
    float m = -INFINITY, l = 0.f;
    v4f o[KC];
#pragma unroll
    for (int dt = 0; dt < KC; ++dt) o[dt] = (v4f){0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < SKP / 16; ++kt) {
      v4f s = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) s = mma(ld4(kb + (kt * 16 + l16) * DP + kc * 16 + 4 * g), qf[kc], s);
      float sv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) sv[i] = (kt * 16 + 4 * g + i < SK) ? s[i] * scale : -INFINITY;
      float tmax = fmaxf(fmaxf(sv[0], sv[1]), fmaxf(sv[2], sv[3]));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mn = fmaxf(m, tmax);
      const float alpha = __expf(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) o[dt] *= alpha;
      float pv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) { pv[i] = __expf(sv[i] - m); l += pv[i]; }
      const s4 pf = pack4(pv[0], pv[1], pv[2], pv[3]);
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) o[dt] = mma(ld4(vb + (dt * 16 + l16) * SKP + kt * 16 + 4 * g), pf, o[dt]);
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.f / l;
    if (qv) {
      bf16_t* op = (bf16_t*)p.o + ((long)b * SQ + q) * p.ldo + h * DH;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < DH) {
          uint2 w;
          w.x = pack2(o[dt][0] * inv, o[dt][1] * inv);
          w.y = pack2(o[dt][2] * inv, o[dt][3] * inv);
          *(uint2*)(op + d0) = w;
        }
      }
      if (g == 0 && p.lse) p.lse[(long)bh * SQ + q] = m + __logf(l);
    }
  }
}

template <int DH>
__global__ __launch_bounds__(256) void attn_bwd_mfma(const EncdiffAttnArgs p, int hpb) {
  constexpr int DP = DH < 16 ? 16 : DH;
  constexpr int KC = DP / 16;
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  const int H = p.heads, SQ = p.sq, SK = p.sk;
  const int SQP = (SQ + 15) & ~15, SKP = (SK + 15) & ~15;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  const int bh0 = blockIdx.x * hpb;
  // per head: Q, dO [SQP][DP]; Qt, dOt [DP][SQP]; K, V [SKP][DP]; Kt [DP][SKP]; lse, D [SQP] fp32
  const int QE = SQP * DP, KE = SKP * DP;
  const int per_head = 4 * QE + 3 * KE;
  float* fls = (float*)(sm + hpb * per_head);
  for (int hl = 0; hl < hpb; ++hl) {
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    bf16_t* base = sm + hl * per_head;
    stage_rows<DH, DP>((const bf16_t*)p.q + (long)b * SQ * p.ldq + h * DH, p.ldq, SQ, SQP, base, base + QE, tid, 256);
    stage_rows<DH, DP>((const bf16_t*)p.d_o + (long)b * SQ * p.lddo + h * DH, p.lddo, SQ, SQP, base + 2 * QE,
                       base + 3 * QE, tid, 256);
    stage_rows<DH, DP>((const bf16_t*)p.k + (long)b * SK * p.ldk + h * DH, p.ldk, SK, SKP, base + 4 * QE,
                       base + 4 * QE + 2 * KE, tid, 256);
    stage_rows<DH, DP>((const bf16_t*)p.v + (long)b * SK * p.ldv + h * DH, p.ldv, SK, SKP, base + 4 * QE + KE,
                       nullptr, tid, 256);
    for (int q = tid; q < SQP; q += 256) {
      float lse = 0.f, D = 0.f;
      if (q < SQ) {
        lse = p.lse[(long)bh * SQ + q];
        const bf16_t* op = (const bf16_t*)p.o + ((long)b * SQ + q) * p.ldo + h * DH;
        const bf16_t* gp = (const bf16_t*)p.d_o + ((long)b * SQ + q) * p.lddo + h * DH;
        for (int d = 0; d < DH; d += 8) {
          float a[8], c[8];
          unpack8(*(const uint4*)(op + d), a);
          unpack8(*(const uint4*)(gp + d), c);
#pragma unroll
          for (int k = 0; k < 8; ++k) D += a[k] * c[k];
        }
      }
      fls[hl * 2 * SQP + q] = lse;
      fls[hl * 2 * SQP + SQP + q] = D;
    }
  }
  __syncthreads();
  const float scale = p.scale;
  const int qtiles = SQP >> 4, ktiles = SKP >> 4;
  // ---- phase A: dK, dV (waves own key tiles) --------------------------------------
  for (int task = wave; task < hpb * ktiles; task += 4) {
    const int hl = task / ktiles, kt = task - hl * ktiles;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    const bf16_t* base = sm + hl * per_head;
    const bf16_t *Qs = base, *Qt = base + QE, *Gs = base + 2 * QE, *Gt = base + 3 * QE;
    const bf16_t *Ks = base + 4 * QE, *Vs = base + 4 * QE + KE;
    const float* lse = fls + hl * 2 * SQP;
    const float* Dv = lse + SQP;
    const int key = kt * 16 + l16;
    const bool kv = key < SK;
    s4 kf[KC], vf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      kf[kc] = ld4(Ks + key * DP + kc * 16 + 4 * g);
      vf[kc] = ld4(Vs + key * DP + kc * 16 + 4 * g);
    }
    v4f dk[KC], dv[KC];
#pragma unroll
    for (int dt = 0; dt < KC; ++dt) { dk[dt] = (v4f){0.f, 0.f, 0.f, 0.f}; dv[dt] = dk[dt]; }
    for (int qt = 0; qt < qtiles; ++qt) {
      v4f s = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        s = mma(ld4(Qs + (qt * 16 + l16) * DP + kc * 16 + 4 * g), kf[kc], s);
        dp = mma(ld4(Gs + (qt * 16 + l16) * DP + kc * 16 + 4 * g), vf[kc], dp);
      }
      float pv[4], ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = qt * 16 + 4 * g + i;
        pv[i] = (kv && q < SQ) ? __expf(s[i] * scale - lse[q]) : 0.f;
        ds[i] = pv[i] * (dp[i] - Dv[q]);
      }
      const s4 pf = pack4(pv[0], pv[1], pv[2], pv[3]);
      const s4 df = pack4(ds[0], ds[1], ds[2], ds[3]);
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) {
        dv[dt] = mma(ld4(Gt + (dt * 16 + l16) * SQP + qt * 16 + 4 * g), pf, dv[dt]);
        dk[dt] = mma(ld4(Qt + (dt * 16 + l16) * SQP + qt * 16 + 4 * g), df, dk[dt]);
      }
    }
    if (kv) {
      bf16_t* dkp = (bf16_t*)p.dk + ((long)b * SK + key) * p.lddk + h * DH;
      bf16_t* dvp = (bf16_t*)p.dv + ((long)b * SK + key) * p.lddv + h * DH;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < DH) {
          uint2 w;
          w.x = pack2(dk[dt][0] * scale, dk[dt][1] * scale);
          w.y = pack2(dk[dt][2] * scale, dk[dt][3] * scale);
          *(uint2*)(dkp + d0) = w;
          w.x = pack2(dv[dt][0], dv[dt][1]);
          w.y = pack2(dv[dt][2], dv[dt][3]);
          *(uint2*)(dvp + d0) = w;
        }
      }
    }
  }
  // ---- phase B: dQ (waves own query tiles) ----------------------------------------
  for (int task = wave; task < hpb * qtiles; task += 4) {
    const int hl = task / qtiles, qt = task - hl * qtiles;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    const bf16_t* base = sm + hl * per_head;
    const bf16_t *Qs = base, *Gs = base + 2 * QE;
    const bf16_t *Ks = base + 4 * QE, *Vs = base + 4 * QE + KE, *Kt = base + 4 * QE + 2 * KE;
    const float* lse = fls + hl * 2 * SQP;
    const float* Dv = lse + SQP;
    const int q = qt * 16 + l16;
    const bool qv = q < SQ;
    const float lq = lse[q], Dq = Dv[q];
    s4 qf[KC], gf[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      qf[kc] = ld4(Qs + q * DP + kc * 16 + 4 * g);
      gf[kc] = ld4(Gs + q * DP + kc * 16 + 4 * g);
    }
    v4f dq[KC];
#pragma unroll
    for (int dt = 0; dt < KC; ++dt) dq[dt] = (v4f){0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < ktiles; ++kt) {
      v4f st = {0.f, 0.f, 0.f, 0.f}, dpt = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        st = mma(ld4(Ks + (kt * 16 + l16) * DP + kc * 16 + 4 * g), qf[kc], st);
        dpt = mma(ld4(Vs + (kt * 16 + l16) * DP + kc * 16 + 4 * g), gf[kc], dpt);
      }
      float ds[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kt * 16 + 4 * g + i;
        const float pr = (qv && key < SK) ? __expf(st[i] * scale - lq) : 0.f;
        ds[i] = pr * (dpt[i] - Dq);
      }
      const s4 df = pack4(ds[0], ds[1], ds[2], ds[3]);
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) dq[dt] = mma(ld4(Kt + (dt * 16 + l16) * SKP + kt * 16 + 4 * g), df, dq[dt]);
    }
    if (qv) {
      bf16_t* dqp = (bf16_t*)p.dq + ((long)b * SQ + q) * p.lddq + h * DH;
#pragma unroll
      for (int dt = 0; dt < KC; ++dt) {
        const int d0 = dt * 16 + 4 * g;
        if (d0 < DH) {
          uint2 w;
          w.x = pack2(dq[dt][0] * scale, dq[dt][1] * scale);
          w.y = pack2(dq[dt][2] * scale, dq[dt][3] * scale);
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

template <int DH>
int launch_mfma_fwd(const EncdiffAttnArgs& a, hipStream_t s) {
  constexpr int DP = DH < 16 ? 16 : DH;
  const int hpb = mfma_hpb(a);
  const int SKP = (a.sk + 15) & ~15;
  const int nblk = a.batch * a.heads / hpb;
  const size_t lds = (size_t)hpb * 2 * SKP * DP * sizeof(bf16_t);
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr = hipFuncSetAttribute((const void*)attn_fwd_mfma<DH>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  hipLaunchKernelGGL(attn_fwd_mfma<DH>, dim3(nblk), dim3(256), lds, s, a, hpb);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

template <int DH>
int launch_mfma_bwd(const EncdiffAttnArgs& a, hipStream_t s) {
  constexpr int DP = DH < 16 ? 16 : DH;
  const int hpb = mfma_hpb(a);
  const int SQP = (a.sq + 15) & ~15, SKP = (a.sk + 15) & ~15;
  const int nblk = a.batch * a.heads / hpb;
  const size_t lds = (size_t)hpb * ((4 * SQP + 3 * SKP) * DP * sizeof(bf16_t) + 2 * SQP * sizeof(float));
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr = hipFuncSetAttribute((const void*)attn_bwd_mfma<DH>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  (void)attr;
  hipLaunchKernelGGL(attn_bwd_mfma<DH>, dim3(nblk), dim3(256), lds, s, a, hpb);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

}  // namespace

// used by attn.hip's dispatcher
int encdiff_attention_mfma(const EncdiffAttnArgs* a, bool bwd, void* stream) {
  if (a->batch * a->heads % mfma_hpb(*a)) return ENCDIFF_ERR_SHAPE;
  hipStream_t s = (hipStream_t)stream;
  switch (a->dh) {
    case 8: return bwd ? launch_mfma_bwd<8>(*a, s) : launch_mfma_fwd<8>(*a, s);
    case 16: return bwd ? launch_mfma_bwd<16>(*a, s) : launch_mfma_fwd<16>(*a, s);
    case 32: return bwd ? launch_mfma_bwd<32>(*a, s) : launch_mfma_fwd<32>(*a, s);
    case 128:  // single-head AttnBlock of the VQ encoder (model.py AttnBlock): forward only (frozen)
      return bwd ? ENCDIFF_ERR_UNSUPPORTED : launch_mfma_fwd<128>(*a, s);
    default: return ENCDIFF_ERR_UNSUPPORTED;
  }
}
