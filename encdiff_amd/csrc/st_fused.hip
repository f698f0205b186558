// st_fused.hip -- the row-local tail of a SpatialTransformer block as one kernel.
//
// After its self-attention, a SpatialTransformer (attention.py:196-261) only mixes channels of
// a token row (projections, LayerNorms, GEGLU) or attends to the 20 concept tokens of the row's
// own image: no row needs another row.  A workgroup therefore keeps R rows resident in LDS --
// the residual stream in fp32, one bf16 operand buffer for the next MFMA -- and runs
//   t1 = o1 Wout1^T + b + t0          (attn1.to_out, residual)
//   n2 = LN2(t1);  q2 = n2 Wq^T        (norm2, attn2.to_q)
//   o2 = softmax(q2 k2^T * scale) v2   (attn2 over the image's concept tokens)
//   t2 = o2 Wout2^T + b + t1          (attn2.to_out, residual)
//   n3 = LN3(t2); [v|g] = n3 W1^T + b; a = v * gelu(g)   (norm3, GEGLU proj, 64-column chunks)
//   t3 = a W2^T + b + t2              (ff.net.2, residual)
//   out = t3 Wpo^T + b + x            (proj_out, block residual)
// with every weight streamed from L2 straight into MFMA B fragments (v_mfma_f32_16x16x32_bf16,
// 4 waves, each owning a quarter of the output columns for all R rows).  Seven launches of the
// unfused path (3 GEMM+LN, to_q, cross-attention, GEGLU proj, ff2 + proj_out -- each a few us of
// launch and load latency at sampling batches) become one.  The training forward additionally
// writes the activations its backward reads (save_*).
#include "common.h"
#include "st_common.h"

#ifndef ED_HEAD64_R32
#define ED_HEAD64_R32 0  // A/B: the c = 64 head on 32-row tiles at training batches
#endif
#ifndef ED_HEAD128_R32
#define ED_HEAD128_R32 1
#endif
#ifndef ED_HEAD128_NWV
#define ED_HEAD128_NWV 4  // waves of the c = 128 head at sampling tiles (8: DDIM 717.8 vs 716.9, no change)
#endif

namespace {

template <int C, int RR>
struct Tail {
  static constexpr int R = RR;                  // rows per workgroup (64; 32 at C = 256: LDS 108 KiB; 16 for tiny batches)
  static constexpr int TM = R / 16;             // 16-row MFMA tiles
  static constexpr int LDT = C + 4;             // fp32 residual-stream row stride (floats)
  static constexpr int LDX = C + 8;             // bf16 operand row stride (elements): conflict-free b128 reads
  static constexpr int NT = C / 64;             // 16-column MFMA tiles per wave for N = C
  static constexpr int HC = 64;                 // GEGLU hidden chunk (columns of a)
  static constexpr int DH = C / 8;              // head dim (8 heads)
  static size_t lds_bytes(int nimg, int nctx) {
    return (size_t)R * LDT * 4 + 2 * (size_t)R * LDX * 2 + (size_t)nimg * 2 * nctx * C * 2;
  }
};

template <int C, int RR, int NWV>
__global__ __launch_bounds__(64 * NWV) void st_tail_kernel(const EncdiffStTailArgs p) {
  using T = Tail<C, RR>;
  // NWV waves: each owns C / NWV output columns of every GEMM and 16 columns of each hidden chunk
  // (8 waves at c = 128: two waves per SIMD hide each other's latencies)
  constexpr int NTH = 64 * NWV, NT = C / (16 * NWV), HC = 16 * NWV;
  constexpr int R = T::R, TM = T::TM, LDT = T::LDT, LDX = T::LDX, DH = T::DH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* Tr = (float*)smem_raw;
  bf16_t* Xa = (bf16_t*)(Tr + R * LDT);
  bf16_t* Xb = Xa + R * LDX;
  bf16_t* KV = Xb + R * LDX;  // [nimg][2][n_ctx][C]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * R;
  const int nctx = p.n_ctx;
  const int img0 = row0 / p.tokens;
  const int nimg = R > p.tokens ? R / p.tokens : 1;
  const bool save = p.save_t1 != nullptr;
  const int n0 = wave * (C / NWV);  // this wave's output columns for N = C

  // Weights.  PRE (c = 64: 128 VGPRs for all of them): every weight fragment of the chain is
  // loaded here, before anything else, so the chain's stages never wait on L2 / MALL latency.
  // c = 128: the four projections here, the feed-forward's chunks double-buffered one chunk
  // ahead; c = 256: each projection while the previous stage runs.
  constexpr int NCH = 4 * C / HC;  // GEGLU hidden chunks
  constexpr bool PRE = C == 64 && NWV == 4;
  constexpr bool PREP = C <= 128;
  constexpr int NW = PRE ? NCH : 2;
  const bf16_t* W1 = (const bf16_t*)p.w_ff1;
  const bf16_t* W2 = (const bf16_t*)p.w_ff2;
  const int nc16 = wave * 16;  // this wave's 16 columns of a hidden chunk
  BFrags<NT, C> wo1, wq, wo2, wpo;
  BFrags<1, C> wv[NW], wg[NW];
  BFrags<NT, HC> w2[PRE ? NCH : 1];
  load_b(wo1, (const bf16_t*)p.w_out1, p.ld_out1, n0, 0, lane);
  if constexpr (PREP) {
    load_b(wq, (const bf16_t*)p.w_q2, p.ld_q2, n0, 0, lane);
    load_b(wo2, (const bf16_t*)p.w_out2, p.ld_out2, n0, 0, lane);
  }
  if constexpr (PRE) {
#pragma unroll
    for (int ch = 0; ch < NW; ++ch) {
      load_b(wv[ch], W1, p.ld_ff1, ch * HC + nc16, 0, lane);
      load_b(wg[ch], W1, p.ld_ff1, 4 * C + ch * HC + nc16, 0, lane);
      load_b(w2[ch], W2, p.ld_ff2, n0, ch * HC, lane);
    }
  }
  if constexpr (PREP) load_b(wpo, (const bf16_t*)p.w_po, p.ld_po, n0, 0, lane);

  // ---- stage: o1 -> Xa, t0 -> Tr (fp32), the tile's concept-token K / V -> LDS
  rows_to_lds<C, R, NTH>(Xa, LDX, (const bf16_t*)p.o1 + (long)row0 * p.ld_o1, p.ld_o1, tid);
  {
    constexpr int CH = C / 8;
    const bf16_t* t0 = (const bf16_t*)p.t0 + (long)row0 * p.ld_t0;
    for (int e = tid; e < R * CH; e += NTH) {
      const int r = e / CH, c8 = (e - r * CH) * 8;
      float f[8];
      unpack8(*(const uint4*)(t0 + (long)r * p.ld_t0 + c8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) Tr[r * LDT + c8 + k] = f[k];
    }
    const int nkv = nimg * 2 * nctx * CH;
    for (int e = tid; e < nkv; e += NTH) {
      const int c8 = (e % CH) * 8, rr = e / CH;  // rr = (i * 2 + kv) * nctx + j
      const int j = rr % nctx, ikv = rr / nctx, kv = ikv & 1, i = ikv >> 1;
      const bf16_t* src = (const bf16_t*)(kv ? p.v2 : p.k2) + (long)((img0 + i) * nctx + j) * p.ld_kv + c8;
      *(uint4*)(KV + (long)rr * C + c8) = *(const uint4*)src;
    }
  }
  __syncthreads();

  v4f acc[TM][NT];
  // ---- t1 = o1 Wout1^T + b + t0
  zero(acc);
  mma(acc, Xa, LDX, wo1, lane);
  if constexpr (!PREP) load_b(wq, (const bf16_t*)p.w_q2, p.ld_q2, n0, 0, lane);  // next GEMM's weights in flight
  acc_add_tr(acc, Tr, LDT, p.b_out1, n0, lane);
  __syncthreads();
  // ---- n2 = LN2(t1)
  if (!(p.pad_ & 4))
  ln_rows<C, R, NTH>(Tr, LDT, Xa, LDX, p.g2, p.be2, p.ln_eps, tid,
                save ? (bf16_t*)p.save_n2 + (long)row0 * p.ld_save : nullptr, p.ld_save,
                save ? (bf16_t*)p.save_t1 + (long)row0 * p.ld_save : nullptr, save ? p.save_s2 + 2L * row0 : nullptr);
  __syncthreads();
  // ---- q2 = n2 Wq^T -> Xb
  zero(acc);
  mma(acc, Xa, LDX, wq, lane);
  if constexpr (!PREP) load_b(wo2, (const bf16_t*)p.w_out2, p.ld_out2, n0, 0, lane);
  acc_store_bf(acc, Xb, LDX, n0, lane);
  __syncthreads();
  if (save) rows_to_global<C, R, NTH>((bf16_t*)p.save_q2 + (long)row0 * p.ld_save, p.ld_save, Xb, LDX, tid);
  // ---- o2 = softmax(q2 k2^T * scale) v2 per (row, head) -> Xa (online softmax over the keys)
  const int dbg = p.pad_;  // timing experiments only (tools/st_tail_bench.py): bit 0 skips the
                           // cross-attention, bit 1 the feed-forward, bit 2 the LayerNorms
  // SPL lanes per (row, head) pair when the workgroup has lanes to spare (sampling tiles): each
  // takes every SPL-th key, the partial softmax states (m, l, o) are merged by lane shuffles
  constexpr int NPR = R * 8;
  constexpr int SPL = NTH / NPR >= 4 ? 4 : (NTH / NPR >= 2 ? 2 : 1);
  const int part = tid % SPL;
  for (int pr = (dbg & 1) ? NPR : tid / SPL; pr < NPR; pr += NTH / SPL) {
    const int r = pr % R, h = pr / R;
    const int il = (row0 + r) / p.tokens - img0;
    // two passes over the keys (all of them are in LDS): the scaled scores' max, then p = exp(s - m)
    // with the scores recomputed bit-identically -- one exp per key and no rescale of o; the dot
    // products on v_dot2_f32_bf16 (bf16 pairs as stored), o accumulated as packed fp32 pairs
    constexpr int DP = DH / 2;
    unsigned qv[DP];
#pragma unroll
    for (int d8 = 0; d8 < DH; d8 += 8) {
      const uint4 a = *(const uint4*)(Xb + r * LDX + h * DH + d8);
      qv[d8 / 2] = a.x; qv[d8 / 2 + 1] = a.y; qv[d8 / 2 + 2] = a.z; qv[d8 / 2 + 3] = a.w;
    }
    const bf16_t* Ks = KV + (long)(il * 2) * nctx * C + h * DH;
    const bf16_t* Vs = Ks + (long)nctx * C;
    auto score = [&](int j) {
      unsigned kv[DP];
#pragma unroll
      for (int d8 = 0; d8 < DH; d8 += 8) {
        const uint4 a = *(const uint4*)(Ks + j * C + d8);
        kv[d8 / 2] = a.x; kv[d8 / 2 + 1] = a.y; kv[d8 / 2 + 2] = a.z; kv[d8 / 2 + 3] = a.w;
      }
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int i = 0; i < DP; i += 2) {
        s0 = dot2bf(qv[i], kv[i], s0);
        s1 = dot2bf(qv[i + 1], kv[i + 1], s1);
      }
      return (s0 + s1) * p.scale;
    };
    float m = -INFINITY, l = 0.f;
#pragma unroll 4
    for (int j = part; j < nctx; j += SPL) m = fmaxf(m, score(j));
    v2f o2[DP];
#pragma unroll
    for (int i = 0; i < DP; ++i) o2[i] = (v2f){0.f, 0.f};
#pragma unroll 2
    for (int j = part; j < nctx; j += SPL) {
      const float pe = __expf(score(j) - m);
      l += pe;
#pragma unroll
      for (int d8 = 0; d8 < DH; d8 += 8) {
        const uint4 b = *(const uint4*)(Vs + j * C + d8);
        const unsigned vv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          o2[d8 / 2 + k] += pe * (v2f){__uint_as_float(vv[k] << 16), __uint_as_float(vv[k] & 0xffff0000u)};
      }
    }
    float o[DH];
#pragma unroll
    for (int i = 0; i < DP; ++i) {
      o[2 * i] = o2[i].x;
      o[2 * i + 1] = o2[i].y;
    }
    if constexpr (SPL > 1) {
#pragma unroll
      for (int off = 1; off < SPL; off <<= 1) {
        const float m2 = __shfl_xor(m, off, 64), l2 = __shfl_xor(l, off, 64);
        const float mx = fmaxf(m, m2);
        const float a = mx == -INFINITY ? 0.f : __expf(m - mx), b = mx == -INFINITY ? 0.f : __expf(m2 - mx);
        l = l * a + l2 * b;
#pragma unroll
        for (int d = 0; d < DH; ++d) o[d] = o[d] * a + __shfl_xor(o[d], off, 64) * b;
        m = mx;
      }
    }
    if (part == 0) {
      const float il_ = 1.f / l;
#pragma unroll
      for (int d8 = 0; d8 < DH; d8 += 8) {
        float y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) y[k] = o[d8 + k] * il_;
        *(uint4*)(Xa + r * LDX + h * DH + d8) = pack8(y);
      }
      if (save) p.save_lse2[(long)((img0 + il) * 8 + h) * p.tokens + (row0 + r) % p.tokens] = m + __logf(l);
    }
  }
  __syncthreads();
  if (save) rows_to_global<C, R, NTH>((bf16_t*)p.save_o2 + (long)row0 * p.ld_save, p.ld_save, Xa, LDX, tid);
  // ---- t2 = o2 Wout2^T + b + t1
  zero(acc);
  mma(acc, Xa, LDX, wo2, lane);
  acc_add_tr(acc, Tr, LDT, p.b_out2, n0, lane);
  __syncthreads();
  // ---- n3 = LN3(t2)  (head mode: t2 / n3 to the caller's buffers, the feed-forward is theirs)
  const bool head = p.head_n3 != nullptr;
  if (!(dbg & 4))
  ln_rows<C, R, NTH>(Tr, LDT, Xa, LDX, p.g3, p.be3, p.ln_eps, tid,
                save ? (bf16_t*)p.save_n3 + (long)row0 * p.ld_save
                     : (head ? (bf16_t*)p.head_n3 + (long)row0 * p.ld_head : nullptr),
                save ? p.ld_save : p.ld_head,
                save ? (bf16_t*)p.save_t2 + (long)row0 * p.ld_save
                     : (head ? (bf16_t*)p.head_t2 + (long)row0 * p.ld_head : nullptr),
                save ? p.save_s3 + 2L * row0 : nullptr);
  if (head) return;
  // ---- GEGLU feed-forward in 64-column chunks of the hidden a; t3 accumulates in registers
  if constexpr (!PRE) {
    load_b(wv[0], W1, p.ld_ff1, nc16, 0, lane);
    load_b(wg[0], W1, p.ld_ff1, 4 * C + nc16, 0, lane);
  }
  __syncthreads();
  v4f acc3[TM][NT];
  zero(acc3);
#pragma unroll
  for (int ch = 0; ch < ((dbg & 2) ? 0 : NCH); ++ch) {
    const int w = PRE ? ch : (ch & 1);  // static after the full unroll
    const int w2i = PRE ? ch : 0;
    if constexpr (!PRE) {
      // this chunk's ff2 fragments and the next chunk's value / gate fragments are in flight
      // while this chunk's value / gate GEMMs and GELU run
      load_b(w2[0], W2, p.ld_ff2, n0, ch * HC, lane);
      if (ch + 1 < NCH) {
        load_b(wv[w ^ 1], W1, p.ld_ff1, (ch + 1) * HC + nc16, 0, lane);
        load_b(wg[w ^ 1], W1, p.ld_ff1, 4 * C + (ch + 1) * HC + nc16, 0, lane);
      }
      if (ch + 1 == NCH && !PREP) load_b(wpo, (const bf16_t*)p.w_po, p.ld_po, n0, 0, lane);
    }
    v4f av[TM][1], ag[TM][1];
    zero(av);
    zero(ag);
    mma(av, Xa, LDX, wv[w], lane);
    mma(ag, Xa, LDX, wg[w], lane);
    {
      const int l16 = lane & 15, g4 = lane >> 4;
      const int col = ch * HC + nc16 + l16;  // hidden column
      const float bvv = p.b_ff1[col], bgg = p.b_ff1[4 * C + col];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 16 * i + 4 * g4 + q;
          const float fv = av[i][0][q] + bvv, fg = ag[i][0][q] + bgg;
          const bf16_t fvb = f2bf(fv), fgb = f2bf(fg);
          // the unfused path stores f in bf16 and forms a from the stored values
          const float y = bf2f(fvb) * gelu_fast(bf2f(fgb));
          Xb[r * LDX + nc16 + l16] = f2bf(y);
          if (save) {
            bf16_t* f = (bf16_t*)p.save_f + (long)(row0 + r) * (8 * C);
            f[col] = fvb;
            f[4 * C + col] = fgb;
            ((bf16_t*)p.save_a)[(long)(row0 + r) * (4 * C) + col] = f2bf(y);
          }
        }
    }
    __syncthreads();
    mma(acc3, Xb, LDX, w2[w2i], lane);
    __syncthreads();  // Xb is rewritten by the next chunk
  }
  // ---- t3 = a W2^T + b + t2;  Xa = bf16(t3);  Tr = x
  acc_add_tr(acc3, Tr, LDT, p.b_ff2, n0, lane);
  __syncthreads();
  {
    constexpr int CH = C / 8;
    const bf16_t* xg = (const bf16_t*)p.x + (long)row0 * p.ld_x;
    for (int e = tid; e < R * CH; e += NTH) {
      const int r = e / CH, c8 = (e - r * CH) * 8;
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = Tr[r * LDT + c8 + k];
      const uint4 t3 = pack8(f);
      *(uint4*)(Xa + r * LDX + c8) = t3;
      if (save) *(uint4*)((bf16_t*)p.save_t3 + (long)(row0 + r) * p.ld_save + c8) = t3;
      unpack8(*(const uint4*)(xg + (long)r * p.ld_x + c8), f);
#pragma unroll
      for (int k = 0; k < 8; ++k) Tr[r * LDT + c8 + k] = f[k];
    }
  }
  __syncthreads();
  // ---- out = t3 Wpo^T + b + x
  zero(acc);
  mma(acc, Xa, LDX, wpo, lane);
  acc_add_tr(acc, Tr, LDT, p.b_po, n0, lane);
  __syncthreads();
  {
    constexpr int CH = C / 8;
    bf16_t* og = (bf16_t*)p.out + (long)row0 * p.ld_out;
    for (int e = tid; e < R * CH; e += NTH) {
      const int r = e / CH, c8 = (e - r * CH) * 8;
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = Tr[r * LDT + c8 + k];
      *(uint4*)(og + (long)r * p.ld_out + c8) = pack8(f);
    }
  }
  if constexpr (R == 64 || R == 32) {
    if (p.gn_stats) {
      // the next GroupNorm's statistics of this 64-row segment (gemm.hip's gn_stats layout): per
      // column sum and sum of squares of the stored bf16 values, TPC row groups added in order;
      // a 32-row tile adds its half of the segment into the zeroed slot (gn_stats_add: with two
      // addends 0 + a + b has the same bits in either order)
      constexpr int TPC = NTH / C, RPG = R / TPC;
      const int col = tid % C, grp = tid / C;
      float a = 0.f, q = 0.f;
#pragma unroll 4
      for (int r = grp * RPG; r < (grp + 1) * RPG; ++r) {
        const float v = bf16_round(Tr[r * LDT + col]);
        a += v;
        q += v * v;
      }
      float* red = (float*)Xa;  // free: the last GEMM read it before the barrier above
      red[grp * C + col] = a;
      red[(TPC + grp) * C + col] = q;
      __syncthreads();
      if (grp == 0) {
        float sa = red[col], sq = red[TPC * C + col];
#pragma unroll
        for (int g = 1; g < TPC; ++g) {
          sa += red[g * C + col];
          sq += red[(TPC + g) * C + col];
        }
        const long slot = row0 >> 6;
        if constexpr (R == 64) {
          p.gn_stats[(2 * slot) * p.ld_gn_stats + col] = sa;
          p.gn_stats[(2 * slot + 1) * p.ld_gn_stats + col] = sq;
        } else {
          atomicAdd(p.gn_stats + (2 * slot) * p.ld_gn_stats + col, sa);
          atomicAdd(p.gn_stats + (2 * slot + 1) * p.ld_gn_stats + col, sq);
        }
      }
    }
  }
}

template <int C, int RR, int NWV>
int launch_tail_w(const EncdiffStTailArgs& p, hipStream_t s) {
  using T = Tail<C, RR>;
  if (p.head_n3 && (!p.head_t2 || p.gn_stats || p.ld_head % 8)) return ENCDIFF_ERR_ARG;
  if (p.rows % T::R || (T::R % p.tokens && p.tokens % T::R)) return ENCDIFF_ERR_SHAPE;
  const int nimg = T::R > p.tokens ? T::R / p.tokens : 1;
  const size_t lds = T::lds_bytes(nimg, p.n_ctx);
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)st_tail_kernel<C, RR, NWV>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr_ok != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)attr_ok;
  hipLaunchKernelGGL((st_tail_kernel<C, RR, NWV>), dim3((unsigned)(p.rows / T::R)), dim3(64 * NWV), lds, s, p);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

// c = 128 with few workgroups (sampling batches): 8 waves per workgroup, two per SIMD hiding each
// other's latencies (B = 8: 24.7 -> 23.3 us); with >= 256 workgroups 4 waves (B = 128: 39 vs 47 us)
template <int C, int RR>
int launch_tail(const EncdiffStTailArgs& p, hipStream_t s) {
  if constexpr (C == 128) {
    if (p.rows / RR < 256) return launch_tail_w<C, RR, 8>(p, s);
  }
  // head mode at c = 256, sampling batches (8 - 128 rows): 8 waves stream the three projections'
  // weights (tools/st_tail_bench.py --head, B=8 4x4: 20.1 -> 18.7 us)
  if constexpr (C == 256 && RR == 16) {
    if (p.head_n3 && p.rows / RR < 256) return launch_tail_w<C, RR, 8>(p, s);
  }
  return launch_tail_w<C, RR, 4>(p, s);
}


// ---------------------------------------------------------------------------------------------
// The head: gn = GroupNorm(x) (from producer segment sums) or read, t0 = proj_in(gn) + b,
// n1 = LN1(t0), qkv = n1 Wqkv^T -- row-local once the GroupNorm statistics are known.
// NWV waves, each owning C / NWV columns of proj_in and of each of the q / k / v column blocks.
// c <= 128 (4 waves): every weight fragment is loaded up front (registers); c = 256 (8 waves,
// sampling tiles of 16 rows): the q / k / v blocks' fragments stream one block ahead.
template <int C, int RR, int NWV>
__global__ __launch_bounds__(64 * NWV) void st_head_kernel(const EncdiffStHeadArgs p) {
  constexpr int NTH = 64 * NWV;
  constexpr int R = RR, TM = R / 16, NT = C / (16 * NWV), LDT = C + 4, LDX = C + 8, LDQ = 3 * C + 8;
  constexpr bool PRE = C <= 128;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* Tr = (float*)smem_raw;
  bf16_t* Xa = (bf16_t*)(Tr + R * LDT);
  bf16_t* Xq = Xa + R * LDX;                          // [R][3C] qkv staging
  float* gms = (float*)(Xq + R * LDQ);                // [nimg][32][2] GroupNorm mean, rstd
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * R;
  const int img0 = row0 / p.tokens;
  const int nimg = R > p.tokens ? R / p.tokens : 1;
  const int n0 = wave * (C / NWV);
  BFrags<NT, C> win;
  BFrags<NT, C> wq[PRE ? 3 : 2];
  load_b(win, (const bf16_t*)p.w_in, p.ld_in, n0, 0, lane);
  if constexpr (PRE) {
#pragma unroll
    for (int j = 0; j < 3; ++j) load_b(wq[j], (const bf16_t*)p.w_qkv, p.ld_w_qkv, j * C + n0, 0, lane);
  }
  constexpr int CH = C / 8;
  if (!p.gn_in_stats && !p.gn) {
    // inference: the statistics of the tile's images from x itself (per channel sum / sum of
    // squares over the image's tokens, thread = (8-channel vector, token lane), lanes and the
    // group's channels added in order), then the same apply as below
    constexpr int cpg = C / 32, NP = NTH / CH;
    float* red = gms + nimg * 64;  // [2][NP][C] scratch behind the statistics (launch_head sizes it)
    const int tv = tid % CH, tp = tid / CH;
    for (int i = 0; i < nimg; ++i) {
      float sa[8], sq[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) sa[k] = sq[k] = 0.f;
      const bf16_t* xb = (const bf16_t*)p.x + (long)(img0 + i) * p.tokens * p.ld_x + tv * 8;
      for (int px0 = tp; px0 < p.tokens; px0 += 8 * NP) {
        uint4 u[8];
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          const int px = px0 + r * NP;
          u[r] = px < p.tokens ? *(const uint4*)(xb + (long)px * p.ld_x) : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          float v[8];
          unpack8(u[r], v);
#pragma unroll
          for (int k = 0; k < 8; ++k) { sa[k] += v[k]; sq[k] += v[k] * v[k]; }
        }
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[tp * C + tv * 8 + k] = sa[k];
        red[(NP + tp) * C + tv * 8 + k] = sq[k];
      }
      __syncthreads();
      if (tid < 32) {
        float a = 0.f, q = 0.f;
        for (int r = 0; r < NP; ++r)
          for (int c = tid * cpg; c < (tid + 1) * cpg; ++c) { a += red[r * C + c]; q += red[(NP + r) * C + c]; }
        const float inv_n = 1.f / ((float)p.tokens * cpg);
        const float mean = a * inv_n;
        gms[2 * (i * 32 + tid)] = mean;
        gms[2 * (i * 32 + tid) + 1] = rsqrtf(fmaxf(q * inv_n - mean * mean, 0.f) + p.gn_eps);
      }
      __syncthreads();
    }
  } else if (p.gn_in_stats) {
    // per (image, group) statistics from the producer's 64-row segment sums (as gn_fwd_stats_kernel)
    constexpr int cpg = C / 32;
    const int nseg = p.tokens >> 6;
    if (tid < nimg * 32) {
      const int i = tid >> 5, g = tid & 31;
      float a = 0.f, q = 0.f;
      for (int sg = 0; sg < nseg; ++sg) {
        const float* st = p.gn_in_stats + 2 * ((long)(img0 + i) * nseg + sg) * p.ld_gn_in_stats + g * cpg;
        for (int c = 0; c < cpg; ++c) {
          a += st[c];
          q += st[p.ld_gn_in_stats + c];
        }
      }
      const float inv_n = 1.f / ((float)p.tokens * cpg);
      const float mean = a * inv_n;
      const float rstd = rsqrtf(fmaxf(q * inv_n - mean * mean, 0.f) + p.gn_eps);
      gms[2 * tid] = mean;
      gms[2 * tid + 1] = rstd;
      if (p.gn_stats && (row0 + i * p.tokens) % p.tokens == 0) {  // this block holds the image's first row
        p.gn_stats[2 * ((long)(img0 + i) * 32 + g)] = mean;
        p.gn_stats[2 * ((long)(img0 + i) * 32 + g) + 1] = rstd;
      }
    }
    __syncthreads();
  }
  if (p.gn_in_stats || !p.gn) {
    constexpr int cpg = C / 32;
    const bf16_t* xg = (const bf16_t*)p.x + (long)row0 * p.ld_x;
    bf16_t* gg = p.gn ? (bf16_t*)p.gn + (long)row0 * p.ld_gn : nullptr;
    for (int e = tid; e < R * CH; e += NTH) {
      const int r = e / CH, c8 = (e - r * CH) * 8, i = (row0 + r) / p.tokens - img0;
      float v[8];
      unpack8(*(const uint4*)(xg + (long)r * p.ld_x + c8), v);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = c8 + k, g = c / cpg;
        const float a = gms[2 * (i * 32 + g) + 1] * p.gn_gamma[c];
        v[k] = v[k] * a + (p.gn_beta[c] - gms[2 * (i * 32 + g)] * a);
      }
      const uint4 y = pack8(v);
      *(uint4*)(Xa + r * LDX + c8) = y;
      if (gg) *(uint4*)(gg + (long)r * p.ld_gn + c8) = y;
    }
  } else {
    rows_to_lds<C, R, NTH>(Xa, LDX, (const bf16_t*)p.gn + (long)row0 * p.ld_gn, p.ld_gn, tid);
  }
  __syncthreads();
  // ---- t0 = gn Win^T + b  (fp32 stream in Tr, bf16 t0 out)
  v4f acc[TM][NT];
  zero(acc);
  mma(acc, Xa, LDX, win, lane);
  if constexpr (!PRE) load_b(wq[0], (const bf16_t*)p.w_qkv, p.ld_w_qkv, n0, 0, lane);  // q block in flight
  {
    const int l16 = lane & 15, g4 = lane >> 4;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = n0 + 16 * j + l16;
      const float bv = p.b_in[col];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) Tr[(16 * i + 4 * g4 + q) * LDT + col] = acc[i][j][q] + bv;
    }
  }
  __syncthreads();
  // ---- n1 = LN1(t0) -> Xa (t0 saved as its bf16 rounding, which the LayerNorm reads)
  ln_rows<C, R, NTH>(Tr, LDT, Xa, LDX, p.g1, p.be1, p.ln_eps, tid,
                     p.n1 ? (bf16_t*)p.n1 + (long)row0 * p.ld_n1 : nullptr, p.ld_n1,
                     p.n1 ? (bf16_t*)p.t0 + (long)row0 * p.ld_t0 : nullptr, p.s1 ? p.s1 + 2L * row0 : nullptr);
  if (!p.n1) {  // inference: t0 is still the tail's residual input
    bf16_t* tg = (bf16_t*)p.t0 + (long)row0 * p.ld_t0;
    for (int e = tid; e < R * CH; e += NTH) {
      const int r = e / CH, c8 = (e - r * CH) * 8;
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = Tr[r * LDT + c8 + k];
      *(uint4*)(tg + (long)r * p.ld_t0 + c8) = pack8(f);
    }
  }
  __syncthreads();
  // ---- qkv = n1 Wqkv^T, one C-column block at a time (staged through LDS for 16-byte stores)
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    if constexpr (!PRE) {
      if (j + 1 < 3) load_b(wq[(j + 1) & 1], (const bf16_t*)p.w_qkv, p.ld_w_qkv, (j + 1) * C + n0, 0, lane);
    }
    v4f aq[TM][NT];
    zero(aq);
    mma(aq, Xa, LDX, wq[PRE ? j : (j & 1)], lane);
    acc_store_bf(aq, Xq, LDQ, j * C + n0, lane);
  }
  __syncthreads();
  rows_to_global<3 * C, R, NTH>((bf16_t*)p.qkv + (long)row0 * p.ld_qkv, p.ld_qkv, Xq, LDQ, tid);
}

template <int C, int RR, int NWV = 4>
int launch_head(const EncdiffStHeadArgs& p, hipStream_t s) {
  constexpr int R = RR;
  if (p.rows % R || (R % p.tokens && p.tokens % R)) return ENCDIFF_ERR_SHAPE;
  const int nimg = R > p.tokens ? R / p.tokens : 1;
  const bool self_stats = !p.gn_in_stats && !p.gn;  // + the statistics scratch [2][NTH / (C / 8)][C] floats
  const size_t lds = (size_t)R * (C + 4) * 4 + (size_t)R * (C + 8) * 2 + (size_t)R * (3 * C + 8) * 2 + nimg * 64 * 4 +
                     (self_stats ? (size_t)64 * 64 * NWV : 0);
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)st_head_kernel<C, RR, NWV>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr_ok != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)attr_ok;
  hipLaunchKernelGGL((st_head_kernel<C, RR, NWV>), dim3((unsigned)(p.rows / R)), dim3(64 * NWV), lds, s, p);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

bool al16(const void* q) { return ((uintptr_t)q & 15) == 0; }

}  // namespace

extern "C" int encdiff_st_tail_fwd(const EncdiffStTailArgs* a, void* stream) {
  if (!a) return ENCDIFF_ERR_ARG;
  const EncdiffStTailArgs& p = *a;
  if (p.heads != 8 || (p.c != 64 && p.c != 128 && p.c != 256)) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.n_ctx < 1 || p.n_ctx > 64 || p.tokens < 1 || p.rows < 1 || p.rows % p.tokens) return ENCDIFF_ERR_SHAPE;
  const void* ptrs[] = {p.o1, p.t0, p.x, p.k2, p.v2, p.w_out1, p.w_q2, p.w_out2, p.w_ff1, p.w_ff2, p.w_po, p.out};
  for (const void* q : ptrs)
    if (!q || !al16(q)) return ENCDIFF_ERR_ARG;
  const long lds[] = {p.ld_o1, p.ld_t0, p.ld_x, p.ld_kv, p.ld_out1, p.ld_q2, p.ld_out2, p.ld_ff1, p.ld_ff2, p.ld_po,
                      p.ld_out};
  for (long l : lds)
    if (l % 8) return ENCDIFF_ERR_ARG;
  if (!p.b_out1 || !p.b_out2 || !p.b_ff1 || !p.b_ff2 || !p.b_po || !p.g2 || !p.be2 || !p.g3 || !p.be3)
    return ENCDIFF_ERR_ARG;
  const void* sv[] = {p.save_t1, p.save_n2, p.save_q2, p.save_o2, p.save_t2, p.save_n3, p.save_f, p.save_a,
                      p.save_t3, p.save_s2, p.save_s3, p.save_lse2};
  int nsave = 0;
  for (const void* q : sv) nsave += q != nullptr;
  // head mode with training saves: the nine activations up to norm3 (the kernel stops there; t2 /
  // n3 go to the save rows, which must be the head rows)
  const bool head_save = p.head_n3 && nsave == 9 && !p.save_f && !p.save_a && !p.save_t3 &&
                         p.save_t2 == p.head_t2 && p.save_n3 == p.head_n3 && p.ld_save == p.ld_head;
  if (nsave != 0 && ((nsave != 12 && !head_save) || p.ld_save % 8)) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  // row tile: 64 rows (32 at c = 256); 16 when the batch is too small for it or the tile's images'
  // concept-token K / V would not fit the LDS (the 2x2 middle block: 4 tokens per image)
  // Few rows (sampling batches): 16-row tiles, so more CUs share the chain (at B = 8 the 64-row
  // tile ran the c = 64 tail in 27 us on 32 CUs, the 16-row tile in 15 us on 128).
  const int rdef = p.c == 256 ? 32 : 64;
  if (p.gn_stats && (p.c == 256 || p.rows % 64 || p.ld_gn_stats < p.c)) return ENCDIFF_ERR_SHAPE;
  int rc = ENCDIFF_ERR_SHAPE;
  // debug mask bit 3: force the 16-row tile; producer statistics need one 64-row tile per segment
  if (p.gn_stats && p.gn_stats_add && p.c == 128 && p.rows / 64 < 256)
    return launch_tail<128, 32>(p, s);  // 8x8 level at B = 128: 256 workgroups instead of 128
  if (p.gn_stats && p.gn_stats_add && p.c == 64) return launch_tail<64, 32>(p, s);  // (ENCDIFF_ST_TAIL_R32_C64)
  if (p.gn_stats || (!(p.pad_ & 8) && p.rows / rdef >= 256))
  switch (p.c) {
    case 64: rc = launch_tail<64, 64>(p, s); break;
    case 128: rc = launch_tail<128, 64>(p, s); break;
    default: rc = launch_tail<256, 32>(p, s); break;
  }
  if (rc != ENCDIFF_ERR_SHAPE || p.gn_stats) return rc;
  switch (p.c) {
    case 64: return launch_tail<64, 16>(p, s);
    case 128: return launch_tail<128, 16>(p, s);
    default: return launch_tail<256, 16>(p, s);
  }
}

extern "C" int encdiff_st_head_fwd(const EncdiffStHeadArgs* a, void* stream) {
  if (!a) return ENCDIFF_ERR_ARG;
  const EncdiffStHeadArgs& p = *a;
  if (p.c != 64 && p.c != 128 && p.c != 256) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.tokens < 1 || p.rows < 1 || p.rows % p.tokens) return ENCDIFF_ERR_SHAPE;
  // c = 256: sampling tiles only (16 rows, 8 waves streaming the weights; a 64-row tile's LDS and
  // the training saves are not provided)
  if (p.c == 256 && (p.rows / 16 >= 256 || p.n1)) return ENCDIFF_ERR_SHAPE;
  if (p.gn_in_stats && (p.tokens % 64 || p.ld_gn_in_stats < p.c || !p.x || !al16(p.x) || p.ld_x % 8))
    return ENCDIFF_ERR_SHAPE;
  const bool self_stats = !p.gn_in_stats && !p.gn;  // statistics from x in the kernel (no gn output)
  if (self_stats && (!p.x || !al16(p.x) || p.ld_x % 8 || p.gn_stats)) return ENCDIFF_ERR_ARG;
  const void* ptrs[] = {self_stats ? p.x : p.gn, p.w_in, p.w_qkv, p.t0, p.qkv};
  for (const void* q : ptrs)
    if (!q || !al16(q)) return ENCDIFF_ERR_ARG;
  const long lds[] = {self_stats ? p.ld_x : p.ld_gn, p.ld_in, p.ld_w_qkv, p.ld_t0, p.ld_qkv};
  for (long l : lds)
    if (l % 8) return ENCDIFF_ERR_ARG;
  if (!p.b_in || !p.g1 || !p.be1 || ((p.gn_in_stats || self_stats) && (!p.gn_gamma || !p.gn_beta)))
    return ENCDIFF_ERR_ARG;
  if ((p.n1 != nullptr) != (p.s1 != nullptr) || (p.n1 && p.ld_n1 % 8)) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  // 64-row tiles at training batches, 16 rows when that leaves most CUs idle (sampling)
  const bool big = p.rows / 64 >= 256;
  int rc = big ? (p.c == 64 ? (ED_HEAD64_R32 ? launch_head<64, 32>(p, s) : launch_head<64, 64>(p, s))
                             : launch_head<128, 64>(p, s))
                : ENCDIFF_ERR_SHAPE;
  if (rc != ENCDIFF_ERR_SHAPE) return rc;
  // c = 128 at the 8x8 training level (8192 rows): 32-row tiles, 256 workgroups (each streams the
  // 128 KB of proj_in + q/k/v weights for twice the rows of a 16-row tile)
  if (ED_HEAD128_R32 && p.c == 128 && p.rows / 32 >= 256) {
    rc = launch_head<128, 32>(p, s);
    if (rc != ENCDIFF_ERR_SHAPE) return rc;
  }
  if (p.c == 256) return launch_head<256, 16, 8>(p, s);
  return p.c == 64 ? launch_head<64, 16>(p, s) : launch_head<128, 16, ED_HEAD128_NWV>(p, s);
}
