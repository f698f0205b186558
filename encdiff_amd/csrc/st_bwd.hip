// st_bwd.hip -- the backward of a SpatialTransformer's row-local parts, one kernel per part.
//
// The forward runs the block's row-local tail (attn1.to_out .. proj_out, attention.py:196-261) as
// st_tail_kernel and its head (GroupNorm .. q/k/v) as st_head_kernel.  Their input-gradient chains
// are row-local too -- every Linear's input gradient, the GEGLU and LayerNorm backwards, and the
// 20-key cross-attention backward of a token row need only that row (plus its image's concept-token
// K / V) -- so a workgroup keeps a tile of R rows in LDS and runs the whole chain:
//
//   st_tail_bwd_kernel:  dy -> d_t3 = dy Wpo -> [64-column GEGLU chunks: d_a = d_t3 W2[:, ch],
//                        d_f = GEGLU'(f) d_a, d_n3 += d_f W1[ch]] -> d_t2 = d_t3 + LN3'(d_n3)
//                        -> d_o2 = d_t2 Wout2 -> cross-attention backward (d_q2, dK2, dV2)
//                        -> d_n2 = d_q2 Wq2 -> d_t1 = d_t2 + LN2'(d_n2) -> d_o1 = d_t1 Wout1
//   st_head_bwd_kernel:  d_qkv -> d_n1 = d_qkv Wqkv -> d_t0 = d_t1 + LN1'(d_n1) -> d_gn = d_t0 Win
//
// The residual-gradient stream stays fp32 in LDS; MFMA operands are bf16 rows in LDS
// (v_mfma_f32_16x16x32_bf16, 4 waves each owning a quarter of the output columns); weights are the
// transposed bf16 copies (B fragments need 8 consecutive reduction elements per lane) streamed from
// L2 one stage ahead.  The gradients the weight-gradient GEMMs read are written out (bf16, as the
// unfused launches store them); the LayerNorm affine partials of a tile are summed over its rows in
// row order (one partial row per workgroup); dK2 / dV2 of an image whose tokens span several tiles
// are written per tile as plain fp32 slabs that st_head_bwd_kernel folds in tile order before it
// uses them (a last-arriver ticket with write-through slabs cost ~7 us per launch).  The weight
// gradients of the block's eight Linears run as ONE grouped launch (st_wgrad_kernel: token-chunk
// partials of every problem, folded in chunk order by st_wgrad_fold_kernel).
#include <algorithm>
#include <cstring>

#include "common.h"
#include "st_common.h"
#include "stwg.h"

namespace {

// GELU and its derivative (erf form) with the branch-free erf of gelu_fast: z = |x| / sqrt(2),
// e = exp(-z^2) = exp(-x^2 / 2) serves both the erf polynomial and the normal density.
ED_DEV void gelu_and_grad(float x, float& g, float& dg) {
  const float z = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * z);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float e = __expf(-z * z);
  const float cdf = 0.5f * (1.f + copysignf(1.f - poly * e, x));
  g = x * cdf;
  dg = cdf + x * (0.39894228040143268f * e);
}

// LayerNorm backward over the R rows of a tile (nn.LayerNorm, attention.py:206-208):
//   xh = (x - mean) rstd,  g = d * gamma,  dx = rstd (g - mean_c(g) - xh mean_c(g xh))
// d (the LayerNorm output gradient) bf16 in LDS, x the saved bf16 input rows and (mean, rstd) the
// saved statistics -- loaded ahead into registers (LnIn, ln_load: TPR lanes per row, NQ 4-channel
// groups per lane).  dx is ADDED to the fp32 residual-gradient stream Tr; the updated stream is
// also written to Xo (bf16 operand).  S receives d * xh per element (the gamma partials' terms).
template <int C, int R, int NTH = 256>
struct LnIn {
  static constexpr int TPR = NTH / R, NQ = C / (4 * TPR);
  uint2 xu[NQ];
  float mean, rstd;
};
template <int C, int R, int NTH = 256>
ED_DEV void ln_load(LnIn<C, R, NTH>& in, const bf16_t* __restrict__ xg, long ldxg, const float* __restrict__ st,
                    int tid) {
  using I = LnIn<C, R, NTH>;
  const int r = tid / I::TPR, k = tid % I::TPR;
#pragma unroll
  for (int i = 0; i < I::NQ; ++i) in.xu[i] = *(const uint2*)(xg + (long)r * ldxg + 4 * (k + I::TPR * i));
  in.mean = st[2 * r];
  in.rstd = st[2 * r + 1];
}
template <int C, int R, int NTH = 256>
ED_DEV void ln_bwd_rows(float* Tr, int ldt, const bf16_t* Dn, int ldx, bf16_t* Xo, const LnIn<C, R, NTH>& in,
                        const float* __restrict__ gamma, float* S, int tid) {
  using I = LnIn<C, R, NTH>;
  constexpr int TPR = I::TPR, NQ = I::NQ;
  const int r = tid / TPR, k = tid % TPR;
  const float mean = in.mean, rstd = in.rstd;
  float xh[NQ][4], gd[NQ][4], s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int c = 4 * (k + TPR * i);
    const uint2 du = *(const uint2*)(Dn + r * ldx + c);
    const float d[4] = {__uint_as_float(du.x << 16), __uint_as_float(du.x & 0xFFFF0000u),
                        __uint_as_float(du.y << 16), __uint_as_float(du.y & 0xFFFF0000u)};
    const float x[4] = {__uint_as_float(in.xu[i].x << 16), __uint_as_float(in.xu[i].x & 0xFFFF0000u),
                        __uint_as_float(in.xu[i].y << 16), __uint_as_float(in.xu[i].y & 0xFFFF0000u)};
    float4 sv;
    float* s = &sv.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xh[i][e] = (x[e] - mean) * rstd;
      gd[i][e] = d[e] * gamma[c + e];
      s1 += gd[i][e];
      s2 += gd[i][e] * xh[i][e];
      s[e] = d[e] * xh[i][e];
    }
    *(float4*)(S + r * ldt + c) = sv;
  }
#pragma unroll
  for (int o = 1; o < TPR; o <<= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  s1 *= (1.f / C);
  s2 *= (1.f / C);
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const int c = 4 * (k + TPR * i);
    float4 t = *(float4*)(Tr + r * ldt + c);
    float* tv = &t.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) tv[e] += rstd * (gd[i][e] - s1 - xh[i][e] * s2);
    *(float4*)(Tr + r * ldt + c) = t;
    *(uint2*)(Xo + r * ldx + c) = make_uint2(pack2(tv[0], tv[1]), pack2(tv[2], tv[3]));
  }
}

// the gamma / beta partial sums of the tile: column c summed over its R rows (S: d * xh fp32, Dn: d
// bf16) -> part row `prow` (2C threads); four interleaved accumulators (rows r mod 4) added in a
// fixed order, so the sum is reproducible and the chain a quarter as long
template <int C, int R>
ED_DEV void ln_partials(const float* S, int ldt, const bf16_t* Dn, int ldx, float* __restrict__ pg,
                        float* __restrict__ pb, long prow, long ld_part, int tid) {
  if (tid < 2 * C) {
    const int c = tid % C;
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (tid < C) {
#pragma unroll 4
      for (int r = 0; r < R; r += 4)
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] += S[(r + i) * ldt + c];
    } else {
#pragma unroll 4
      for (int r = 0; r < R; r += 4)
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] += bf2f(Dn[(r + i) * ldx + c]);
    }
    (tid < C ? pg : pb)[prow * ld_part + c] = (a[0] + a[1]) + (a[2] + a[3]);
  }
}

template <int N>
struct FChunk {
  v4u32 v[N];  // native vectors (HIP's uint4 struct copies kept these arrays in scratch)
};
// thread tid's 16-byte pieces of the f chunk ch: value columns [ch*HC, +HC), gate columns 4C + same
template <int C, int HC, int FCPR, int NTH, int N>
ED_DEV void f_load(FChunk<N>& fr, const bf16_t* __restrict__ F, long ld, int ch, int tid) {
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const int e = tid + u * NTH, r = e / FCPR, c8 = (e % FCPR) * 8;
    const int gc = c8 < HC ? ch * HC + c8 : 4 * C + ch * HC + (c8 - HC);
    fr.v[u] = *(const v4u32*)(F + (long)r * ld + gc);
  }
}

template <int C, int R>
struct TailBwd {
  static constexpr int LDT = C + 4, LDX = C + 8, HC = 64, LDH = 2 * HC + 8;
  static constexpr size_t ubytes() {
    const size_t a = (size_t)R * LDH * 2, b = (size_t)R * LDT * 4, c = (size_t)R * LDX * 2;
    const size_t m = a > b ? (a > c ? a : c) : (b > c ? b : c);
    return (m + 15) / 16 * 16;
  }
  // MF: the per-(row, head) P / dS tiles of one round of heads (NTH / R heads: 256 pairs) for the
  // MFMA key-gradient pass, [2][NTH / R][R][JP] bf16 (JP = n_ctx rounded up to 4), + a 64-B tail the
  // last fragment reads may touch; otherwise per (row, head) LSE / D for the VALU (head, key) pass
  // Layout: Tr | Xa | Xb | KV | U (| AT); the P / dS round starts in U right after the q2 rows the
  // cross-attention keeps there (the rest of U is free during the attention) and may run past U.
  static constexpr int jp(int nctx) { return (nctx + 3) & ~3; }
  static constexpr size_t qbytes() { return (size_t)R * LDX * 2; }
  static size_t lds_bytes(int nctx, bool mf) {
    const size_t ps = (size_t)256 * jp(nctx) * 2 * 2 + 64;
    const size_t u = mf ? std::max(ubytes(), qbytes() + ps) : ubytes() + (size_t)2 * R * 8 * 4;
    return (size_t)R * LDT * 4 + 2 * (size_t)R * LDX * 2 + (size_t)2 * nctx * C * 2 + u + 16;
  }
};

#ifndef ST_BWD_JU
#define ST_BWD_JU 2  // key pairs per iteration of the (row, head) pass (LDS reads of K / V in flight)
#endif
// k-outer fragment (8 consecutive k of column col + l16) of a k-major bf16 tile in LDS: two
// transposed 4 x 16 reads (ds_read_b64_tr_b16); rows g4 * 8 .. + 8 of the tile
ED_DEV v8bf frag_tr(const bf16_t* tile, int ld, int col, int lane) {
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  const int l16 = lane & 15, g4 = lane >> 4, tq = l16 >> 2, tp = l16 & 3;
  const bf16_t* a0 = tile + (g4 * 8 + tq) * ld + col + 4 * tp;
  const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
  const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * ld));
  return __builtin_bit_cast(v8bf, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int C, int R, bool MF>
__global__ __launch_bounds__(256, (C == 128 && R == 64) ? 1 : 2) void st_tail_bwd_kernel(const EncdiffStTailBwdArgs p) {
  using T = TailBwd<C, R>;
  constexpr int NWV = 4, NTH = 256, TM = R / 16, NT = C / (16 * NWV);
  constexpr int LDT = T::LDT, LDX = T::LDX, HC = T::HC, LDH = T::LDH, NCH = 4 * C / HC, DH = C / 8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* Tr = (float*)smem_raw;                          // [R][LDT] fp32 residual-gradient stream
  bf16_t* Xa = (bf16_t*)(Tr + R * LDT);                  // [R][LDX] bf16 operand
  bf16_t* Xb = Xa + R * LDX;                             // [R][LDX] bf16 operand
  const int nctx = p.n_ctx;
  bf16_t* KV = Xb + R * LDX;                             // [2][nctx][C] the image's concept K / V
  unsigned char* U = (unsigned char*)(KV + 2 * nctx * C);  // union: GEGLU chunk | LN terms | q2 rows
  bf16_t* Xh = (bf16_t*)U;                               //   [R][LDH] f chunk -> d_f chunk (value | gate)
  float* S = (float*)U;                                  //   [R][LDT] d * xh of a LayerNorm backward
  bf16_t* Q = (bf16_t*)U;                                //   [R][LDX] q2 rows (cross-attention)
  float* AT = (float*)(U + T::ubytes());                 // [2][R][8]: lse, D per (row, head) (!MF)
  bf16_t* PS = (bf16_t*)(U + T::qbytes());               // [2][NTH / R][R][JP]: P, dS of a head round (MF)

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g4 = lane >> 4;
  const int row0 = blockIdx.x * R;
  const int img = row0 / p.tokens;
  const int n0 = wave * (C / NWV);  // this wave's output columns for N = C
  const int nc16 = wave * 16;       // ... and of a 64-column hidden chunk
  const bf16_t* W2T = (const bf16_t*)p.w_ff2_t;
  const bf16_t* W1T = (const bf16_t*)p.w_ff1_t;
  const bf16_t* F = (const bf16_t*)p.f + (long)row0 * p.ld_f;
  // timing experiments only (tools/st_bwd_bench.py; 0 in every product call): 1 no GEGLU math,
  // 2 no (row, head) attention pass, 4 no (head, key) pass, 8 no LayerNorm math, 16 no gradient
  // stores, 32 the (head, key) pass without its dK / dV stores
  const int dbg = p.pad_;

  // the f chunk (value | gate columns of the 64-column hidden chunk) as 16-byte rows: FCH per thread
  constexpr int FCPR = 2 * HC / 8, FCH = R * FCPR / NTH;
  FChunk<FCH> fr, fn;  // this chunk's f, the next chunk's
  f_load<C, HC, FCPR, NTH>(fr, F, p.ld_f, 0, tid);
  // every saved row input of the later stages is requested now, before the kernel's first global
  // store: vmcnt is one in-order counter for loads and stores, so a load issued after a store
  // cannot be waited for without waiting for that store too.  LN3 / LN2 inputs (t2, t1 rows and
  // statistics), the cross-attention's q2 rows (16-byte chunks) and per (row, head) pair o2 and LSE
  LnIn<C, R, NTH> ln3, ln2;
  ln_load<C, R, NTH>(ln3, (const bf16_t*)p.t2 + (long)row0 * p.ld_save, p.ld_save, p.s3 + 2L * row0, tid);
  ln_load<C, R, NTH>(ln2, (const bf16_t*)p.t1 + (long)row0 * p.ld_save, p.ld_save, p.s2 + 2L * row0, tid);
  constexpr int QCH = R * (C / 8) / NTH, NPR = R * 8, PPT = (NPR + NTH - 1) / NTH, DV = DH / 8;
  v4u32 qr[QCH];
#pragma unroll
  for (int u = 0; u < QCH; ++u) {
    const int e = tid + u * NTH, r = e / (C / 8), c8 = (e % (C / 8)) * 8;
    qr[u] = *(const v4u32*)((const bf16_t*)p.q2 + (long)(row0 + r) * p.ld_save + c8);
  }
  v4u32 o2r[PPT][DV];
  float lse_r[PPT];
#pragma unroll
  for (int u = 0; u < PPT; ++u) {
    const int pr = tid + u * NTH, r = pr % R, h = pr / R;
#pragma unroll
    for (int v = 0; v < DV; ++v)
      o2r[u][v] = *(const v4u32*)((const bf16_t*)p.o2 + (long)(row0 + r) * p.ld_save + h * DH + 8 * v);
    lse_r[u] = p.lse2[(long)(img * 8 + h) * p.tokens + (row0 + r) % p.tokens];
  }

  // weights one stage ahead: proj_out^T now, the first GEGLU chunk's next
  BFrags<NT, C> wp;
  BFrags<1, C> w2, w2n;
  BFrags<NT, HC> w1v, w1g, w1vn, w1gn;
  load_b(wp, (const bf16_t*)p.w_po_t, C, n0, 0, lane);
  load_b(w2, W2T, C, nc16, 0, lane);
  load_b(w1v, W1T, 8 * C, n0, 0, lane);
  load_b(w1g, W1T, 8 * C, n0, 4 * C, lane);

  // ---- stage: dy -> Xa, the image's concept K / V -> LDS
  rows_to_lds<C, R, NTH>(Xa, LDX, (const bf16_t*)p.dy + (long)row0 * p.ld_dy, p.ld_dy, tid);
  {
    constexpr int CH = C / 8;
    for (int e = tid; e < 2 * nctx * CH; e += NTH) {
      const int c8 = (e % CH) * 8, rr = e / CH, j = rr % nctx, kv = rr / nctx;
      *(uint4*)(KV + (long)rr * C + c8) =
          *(const uint4*)((const bf16_t*)(kv ? p.v2 : p.k2) + (long)(img * nctx + j) * p.ld_kv + c8);
    }
  }
  __syncthreads();

  v4f acc[TM][NT];
  // ---- d_t3 = dy Wpo  (residual stream Tr, bf16 operand Xb)
  zero(acc);
  mma(acc, Xa, LDX, wp, lane);
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * i + 4 * g4 + q, col = n0 + 16 * j + l16;
        Tr[r * LDT + col] = acc[i][j][q];
        Xb[r * LDX + col] = f2bf(acc[i][j][q]);
      }
  __syncthreads();
  if (!(dbg & 16)) rows_to_global<C, R, NTH>((bf16_t*)p.d_t3 + (long)row0 * p.ld_d, p.ld_d, Xb, LDX, tid);

  // ---- GEGLU feed-forward backward in 64-column chunks of the hidden a; d_n3 accumulates.
  // Per chunk: the f chunk (prefetched a chunk ahead, 16-byte loads) is staged into Xh, d_a of the
  // wave's 16 hidden columns comes from the MFMA, and each lane turns its (value, gate) pairs of Xh
  // into (d value, d gate) in place; then Xh -> global d_f and d_n3 += Xh W1[chunk].
  v4f acc3[TM][NT];
  zero(acc3);
  BFrags<NT, C> wo2, wq2;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
#pragma unroll
    for (int u = 0; u < FCH; ++u) {
      const int e = tid + u * NTH, r = e / FCPR, c8 = (e % FCPR) * 8;
      *(v4u32*)(Xh + r * LDH + c8) = fr.v[u];
    }
    if (ch + 1 < NCH) {
      f_load<C, HC, FCPR, NTH>(fn, F, p.ld_f, ch + 1, tid);
      load_b(w2n, W2T, C, (ch + 1) * HC + nc16, 0, lane);
      load_b(w1vn, W1T, 8 * C, n0, (ch + 1) * HC, lane);
      load_b(w1gn, W1T, 8 * C, n0, 4 * C + (ch + 1) * HC, lane);
    } else {  // the next stages' weights, issued before this chunk's d_f stores
      load_b(wo2, (const bf16_t*)p.w_out2_t, C, n0, 0, lane);
      load_b(wq2, (const bf16_t*)p.w_q2_t, C, n0, 0, lane);
    }
    v4f av[TM][1];
    zero(av);
    mma(av, Xb, LDX, w2, lane);
    __syncthreads();  // Xh staged
    if (!(dbg & 1)) {
      // the lane's (value, gate) pairs: all loads first, then the math, then the stores
      float a[TM][4], gt[TM][4];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const bf16_t* hv = Xh + (16 * i + 4 * g4 + q) * LDH + nc16 + l16;
          a[i][q] = bf2f(hv[0]);
          gt[i][q] = bf2f(hv[HC]);
        }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          bf16_t* hv = Xh + (16 * i + 4 * g4 + q) * LDH + nc16 + l16;
          const float d = bf16_round(av[i][0][q]);  // d_a as the unfused path stores it
          float gl, dgl;
          gelu_and_grad(gt[i][q], gl, dgl);
          hv[0] = f2bf(d * gl);
          hv[HC] = f2bf(d * a[i][q] * dgl);
        }
    } else {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) Xh[(16 * i + 4 * g4 + q) * LDH + nc16 + l16] = f2bf(av[i][0][q]);
    }
    __syncthreads();
    {  // the chunk's d_f rows -> global (value and gate halves, 16-byte stores)
      bf16_t* dfg = (bf16_t*)p.d_f + (long)row0 * p.ld_df;
      if (!(dbg & 16)) {
#pragma unroll
        for (int u = 0; u < FCH; ++u) {
          const int e = tid + u * NTH, r = e / FCPR, c8 = (e % FCPR) * 8;
          const int gc = c8 < HC ? ch * HC + c8 : 4 * C + ch * HC + (c8 - HC);
          *(uint4*)(dfg + (long)r * p.ld_df + gc) = *(const uint4*)(Xh + r * LDH + c8);
        }
      }
    }
    mma(acc3, Xh, LDH, w1v, lane);
    mma(acc3, Xh + HC, LDH, w1g, lane);
    __syncthreads();  // Xh is rewritten by the next chunk
    if (ch + 1 < NCH) {
#pragma unroll
      for (int u = 0; u < FCH; ++u) fr.v[u] = fn.v[u];
      w2 = w2n;
      w1v = w1vn;
      w1g = w1gn;
    }
  }
  // ---- d_n3 -> Xa (bf16, as stored by the unfused input-gradient GEMM); LN3 backward
  acc_store_bf(acc3, Xa, LDX, n0, lane);
  __syncthreads();
  if (!(dbg & 8)) ln_bwd_rows<C, R, NTH>(Tr, LDT, Xa, LDX, Xb, ln3, p.g3, S, tid);
  __syncthreads();
  ln_partials<C, R>(S, LDT, Xa, LDX, p.ln3_dg, p.ln3_db, blockIdx.x, p.ld_part, tid);
  if (!(dbg & 16)) rows_to_global<C, R, NTH>((bf16_t*)p.d_t2 + (long)row0 * p.ld_d, p.ld_d, Xb, LDX, tid);
  // ---- d_o2 = d_t2 Wout2 -> Xa
  zero(acc);
  mma(acc, Xb, LDX, wo2, lane);
  BFrags<NT, C> wo1;
  load_b(wo1, (const bf16_t*)p.w_out1_t, C, n0, 0, lane);
  __syncthreads();  // (S / Xa readers of the partial sums are done)
  acc_store_bf(acc, Xa, LDX, n0, lane);
#pragma unroll
  for (int u = 0; u < QCH; ++u) {
    const int e = tid + u * NTH, r = e / (C / 8), c8 = (e % (C / 8)) * 8;
    *(v4u32*)(Q + r * LDX + c8) = qr[u];
  }
  __syncthreads();

  const int tpi = p.tokens / R;  // tiles per image
  if constexpr (MF) {
    // ---- cross-attention backward with the key gradients on MFMA.  Per round of HPR = NTH / R heads
    // (one (row, head) pair per thread): D = do . o, p_j = exp(s_j - lse), ds_j = p_j (do . v_j - D),
    // dq = scale sum_j ds_j k_j (VALU, as the forward), P and dS rows -> LDS (bf16, [head][row][key]);
    // then dV_h = P_h^T dO_h and dK_h = scale dS_h^T Q_h as 16 (keys) x 16 (head columns) MFMA tiles
    // over the tile's rows (k), the k-major P / dS and the row-major dO / Q read as k-outer fragments
    // with ds_read_b64_tr_b16.  Key rows >= n_ctx of the last key tile and, at head dim 8, the 8
    // columns of the neighbouring head are computed and dropped.
    constexpr int HPR = NTH / R;
    const int JP = T::jp(nctx), JT = (nctx + 15) / 16;
    bf16_t* Pb = PS;
    bf16_t* Db = PS + HPR * R * JP;
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int r = tid % R, hl = tid / R, h = u * HPR + hl;
      if (!(dbg & 2)) {
        // bf16 pairs as loaded: the dot products on v_dot2_f32_bf16 (fp32 accumulation of the exact
        // bf16 products), dq accumulated as packed fp32 pairs
        constexpr int DP = DH / 2;
        unsigned qv[DP], dov[DP], ov[DP];
#pragma unroll
        for (int v = 0; v < DV; ++v) {
          const uint4 a = *(const uint4*)(Q + r * LDX + h * DH + 8 * v);
          const uint4 b = *(const uint4*)(Xa + r * LDX + h * DH + 8 * v);
          qv[4 * v] = a.x; qv[4 * v + 1] = a.y; qv[4 * v + 2] = a.z; qv[4 * v + 3] = a.w;
          dov[4 * v] = b.x; dov[4 * v + 1] = b.y; dov[4 * v + 2] = b.z; dov[4 * v + 3] = b.w;
#pragma unroll
          for (int k = 0; k < 4; ++k) ov[4 * v + k] = o2r[u][v][k];
        }
        float D = 0.f;
#pragma unroll
        for (int i = 0; i < DP; ++i) D = dot2bf(dov[i], ov[i], D);
        v2f dq[DP];
#pragma unroll
        for (int i = 0; i < DP; ++i) dq[i] = (v2f){0.f, 0.f};
        bf16_t* prow = Pb + (hl * R + r) * JP;
        bf16_t* drow = Db + (hl * R + r) * JP;
#pragma unroll ST_BWD_JU
        for (int j = 0; j < JP; j += 2) {
          float pj[2], ds[2];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int jj = j + e < nctx ? j + e : 0;
            unsigned kv[DP], vv[DP];
#pragma unroll
            for (int v = 0; v < DV; ++v) {
              const uint4 a = *(const uint4*)(KV + jj * C + h * DH + 8 * v);
              const uint4 b = *(const uint4*)(KV + (nctx + jj) * C + h * DH + 8 * v);
              kv[4 * v] = a.x; kv[4 * v + 1] = a.y; kv[4 * v + 2] = a.z; kv[4 * v + 3] = a.w;
              vv[4 * v] = b.x; vv[4 * v + 1] = b.y; vv[4 * v + 2] = b.z; vv[4 * v + 3] = b.w;
            }
            float s0 = 0.f, s1 = 0.f, p0 = 0.f, p1 = 0.f;
#pragma unroll
            for (int i = 0; i < DP; i += 2) {
              s0 = dot2bf(qv[i], kv[i], s0);
              s1 = dot2bf(qv[i + 1], kv[i + 1], s1);
              p0 = dot2bf(dov[i], vv[i], p0);
              p1 = dot2bf(dov[i + 1], vv[i + 1], p1);
            }
            const float pe = j + e < nctx ? __expf((s0 + s1) * p.scale - lse_r[u]) : 0.f;
            pj[e] = pe;
            ds[e] = pe * ((p0 + p1) - D);
#pragma unroll
            for (int i = 0; i < DP; ++i)
              dq[i] += ds[e] * (v2f){__uint_as_float(kv[i] << 16), __uint_as_float(kv[i] & 0xffff0000u)};
          }
          *(unsigned*)(prow + j) = pack2(pj[0], pj[1]);
          *(unsigned*)(drow + j) = pack2(ds[0], ds[1]);
        }
#pragma unroll
        for (int v = 0; v < DV; ++v) {
          float y[8];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            y[2 * k] = dq[4 * v + k].x * p.scale;
            y[2 * k + 1] = dq[4 * v + k].y * p.scale;
          }
          *(uint4*)(Xb + r * LDX + h * DH + 8 * v) = pack8(y);
        }
      }
      __syncthreads();
      // key-gradient tiles of this round: (head, key tile, dV | dK), round-robin over the waves
      for (int t = (dbg & 4) ? HPR * JT * 2 : wave; t < HPR * JT * 2; t += NWV) {
        const int kind = t & 1, jt = (t >> 1) % JT, hh = (t >> 1) / JT, hg = u * HPR + hh;
        const bf16_t* A = (kind ? Db : Pb) + hh * R * JP;
        const bf16_t* B = kind ? Q : Xa;
        v4f a = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < R / 32; ++ks)
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(A + 32 * ks * JP, JP, 16 * jt, lane),
                                                      frag_tr(B + 32 * ks * LDX, LDX, hg * DH, lane), a, 0, 0, 0);
        const int d = l16;
        if (d < DH && !(dbg & 32)) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int j = 16 * jt + 4 * g4 + q;
            if (j >= nctx) continue;
            const float val = kind ? a[q] * p.scale : a[q];
            if (tpi == 1) {
              bf16_t* dst = (bf16_t*)(kind ? p.dk2 : p.dv2) + (long)(img * nctx + j) * p.ld_dkv + hg * DH + d;
              *dst = f2bf(val);
            } else {  // fp32 partial slab of this tile; encdiff_st_head_bwd folds an image's slabs in tile order
              p.kv_part[((long)blockIdx.x * nctx + j) * 2 * C + (kind ? 0 : C) + hg * DH + d] = val;
            }
          }
        }
      }
      __syncthreads();  // P / dS rewritten by the next round; Xa / Q read by the tiles above
    }
  } else {
  // ---- cross-attention backward (attention.py:180-191 with the softmax recomputed from the LSE):
  // per (row, head): D = do . o, p_j = exp(s_j - lse), ds_j = p_j (do . v_j - D), dq = scale sum ds_j k_j.
  // A thread's PPT pairs run interleaved (independent chains per key).
  if (!(dbg & 2)) {
    static_assert(NPR % NTH == 0, "row-head pairs fill the threads");
    float q[PPT][DH], dout[PPT][DH], dq[PPT][DH], D[PPT];
    int rr[PPT], hh[PPT];
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int pr = tid + u * NTH, r = pr % R, h = pr / R;
      rr[u] = r;
      hh[u] = h;
      float o[DH];
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        unpack8(*(const uint4*)(Q + r * LDX + h * DH + 8 * v), q[u] + 8 * v);
        unpack8(*(const uint4*)(Xa + r * LDX + h * DH + 8 * v), dout[u] + 8 * v);
        unpack8(make_uint4(o2r[u][v][0], o2r[u][v][1], o2r[u][v][2], o2r[u][v][3]), o + 8 * v);
      }
      D[u] = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        D[u] += dout[u][d] * o[d];
        dq[u][d] = 0.f;
      }
    }
#pragma unroll 2
    for (int j = 0; j < nctx; ++j) {
#pragma unroll
      for (int u = 0; u < PPT; ++u) {
        const int h = hh[u];
        float kf[DH], vf[DH];
#pragma unroll
        for (int v = 0; v < DV; ++v) {
          unpack8(*(const uint4*)(KV + j * C + h * DH + 8 * v), kf + 8 * v);
          unpack8(*(const uint4*)(KV + (nctx + j) * C + h * DH + 8 * v), vf + 8 * v);
        }
        float s0 = 0.f, s1 = 0.f, p0 = 0.f, p1 = 0.f;
#pragma unroll
        for (int d = 0; d < DH; d += 2) {
          s0 += q[u][d] * kf[d];
          s1 += q[u][d + 1] * kf[d + 1];
          p0 += dout[u][d] * vf[d];
          p1 += dout[u][d + 1] * vf[d + 1];
        }
        const float pj = __expf((s0 + s1) * p.scale - lse_r[u]);
        const float ds = pj * ((p0 + p1) - D[u]);
#pragma unroll
        for (int d = 0; d < DH; ++d) dq[u][d] += ds * kf[d];
      }
    }
#pragma unroll
    for (int u = 0; u < PPT; ++u) {
      const int r = rr[u], h = hh[u];
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        float y[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) y[k] = dq[u][8 * v + k] * p.scale;
        *(uint4*)(Xb + r * LDX + h * DH + 8 * v) = pack8(y);
      }
      AT[h * R + r] = lse_r[u];  // [head][row]: 4 consecutive rows in one float4 below
      AT[R * 8 + h * R + r] = D[u];
    }
  }
  __syncthreads();
  // dK_j = scale sum_r ds_rj q_r, dV_j = sum_r p_rj do_r over the tile's rows, per (head, key); four
  // rows per step with independent score chains
  {
    for (int t = (dbg & 4) ? 8 * nctx : tid; t < 8 * nctx; t += NTH) {
      const int h = t / nctx, j = t - h * nctx;
      float kf[DH], vf[DH], dk[DH], dv[DH];
#pragma unroll
      for (int v = 0; v < DV; ++v) {
        unpack8(*(const uint4*)(KV + j * C + h * DH + 8 * v), kf + 8 * v);
        unpack8(*(const uint4*)(KV + (nctx + j) * C + h * DH + 8 * v), vf + 8 * v);
      }
#pragma unroll
      for (int d = 0; d < DH; ++d) dk[d] = dv[d] = 0.f;
      constexpr int RU = DH == 8 ? 4 : 2;  // rows per step (register budget at head dim 16)
      for (int r0 = 0; r0 < R; r0 += RU) {
        float lse4[RU], D4[RU];
        if constexpr (RU == 4) {
          const float4 l4 = *(const float4*)(AT + h * R + r0);
          const float4 d4 = *(const float4*)(AT + R * 8 + h * R + r0);
          lse4[0] = l4.x; lse4[1] = l4.y; lse4[2] = l4.z; lse4[3] = l4.w;
          D4[0] = d4.x; D4[1] = d4.y; D4[2] = d4.z; D4[3] = d4.w;
        } else {
          const float2 l2 = *(const float2*)(AT + h * R + r0);
          const float2 d2 = *(const float2*)(AT + R * 8 + h * R + r0);
          lse4[0] = l2.x; lse4[1] = l2.y;
          D4[0] = d2.x; D4[1] = d2.y;
        }
        float q[RU][DH], dout[RU][DH], pj[RU], ds[RU];
#pragma unroll
        for (int i = 0; i < RU; ++i) {
#pragma unroll
          for (int v = 0; v < DV; ++v) {
            unpack8(*(const uint4*)(Q + (r0 + i) * LDX + h * DH + 8 * v), q[i] + 8 * v);
            unpack8(*(const uint4*)(Xa + (r0 + i) * LDX + h * DH + 8 * v), dout[i] + 8 * v);
          }
        }
#pragma unroll
        for (int i = 0; i < RU; ++i) {
          float s = 0.f, dp = 0.f;
#pragma unroll
          for (int d = 0; d < DH; ++d) {
            s += q[i][d] * kf[d];
            dp += dout[i][d] * vf[d];
          }
          pj[i] = __expf(s * p.scale - lse4[i]);
          ds[i] = pj[i] * (dp - D4[i]);
        }
#pragma unroll
        for (int d = 0; d < DH; ++d) {
          if constexpr (RU == 4) {
            dk[d] += (ds[0] * q[0][d] + ds[1] * q[1][d]) + (ds[2] * q[2][d] + ds[3] * q[3][d]);
            dv[d] += (pj[0] * dout[0][d] + pj[1] * dout[1][d]) + (pj[2] * dout[2][d] + pj[3] * dout[3][d]);
          } else {
            dk[d] += ds[0] * q[0][d] + ds[1] * q[1][d];
            dv[d] += pj[0] * dout[0][d] + pj[1] * dout[1][d];
          }
        }
      }
#pragma unroll
      for (int d = 0; d < DH; ++d) dk[d] *= p.scale;
      if (dbg & 32) {  // (timing) the pass's arithmetic without its stores: keep it live
        float sum = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) sum += dk[d] + dv[d];
        if (sum == 12345.f) Tr[0] = sum;
      } else if (tpi == 1) {
#pragma unroll
        for (int v = 0; v < DV; ++v) {
          *(uint4*)((bf16_t*)p.dk2 + (long)(img * nctx + j) * p.ld_dkv + h * DH + 8 * v) = pack8(dk + 8 * v);
          *(uint4*)((bf16_t*)p.dv2 + (long)(img * nctx + j) * p.ld_dkv + h * DH + 8 * v) = pack8(dv + 8 * v);
        }
      } else {  // fp32 partial slab of this tile; encdiff_st_head_bwd folds an image's slabs in tile order
        float* slab = p.kv_part + ((long)blockIdx.x * nctx + j) * 2 * C + h * DH;
#pragma unroll
        for (int d4 = 0; d4 < DH; d4 += 4) {
          *(float4*)(slab + d4) = make_float4(dk[d4], dk[d4 + 1], dk[d4 + 2], dk[d4 + 3]);
          *(float4*)(slab + C + d4) = make_float4(dv[d4], dv[d4 + 1], dv[d4 + 2], dv[d4 + 3]);
        }
      }
    }
  }
  }
  // ---- d_n2 = d_q2 Wq2 -> Xa   (Xb = d_q2 out; Xa's d_o2 rows are read by the dK / dV loop above)
  __syncthreads();
  if (!(dbg & 16)) rows_to_global<C, R, NTH>((bf16_t*)p.d_q2 + (long)row0 * p.ld_d, p.ld_d, Xb, LDX, tid);
  zero(acc);
  mma(acc, Xb, LDX, wq2, lane);
  acc_store_bf(acc, Xa, LDX, n0, lane);
  __syncthreads();
  // ---- LN2 backward: d_t1 = d_t2 + LN2'(t1; d_n2)
  if (!(dbg & 8)) ln_bwd_rows<C, R, NTH>(Tr, LDT, Xa, LDX, Xb, ln2, p.g2, S, tid);
  __syncthreads();
  ln_partials<C, R>(S, LDT, Xa, LDX, p.ln2_dg, p.ln2_db, blockIdx.x, p.ld_part, tid);
  if (!(dbg & 16)) rows_to_global<C, R, NTH>((bf16_t*)p.d_t1 + (long)row0 * p.ld_d, p.ld_d, Xb, LDX, tid);
  // ---- d_o1 = d_t1 Wout1
  zero(acc);
  mma(acc, Xb, LDX, wo1, lane);
  __syncthreads();  // Xa (d_n2) readers are done
  acc_store_bf(acc, Xa, LDX, n0, lane);
  __syncthreads();
  if (!(dbg & 16)) rows_to_global<C, R, NTH>((bf16_t*)p.d_o1 + (long)row0 * p.ld_d, p.ld_d, Xa, LDX, tid);
}

// the MFMA key-gradient form where its P / dS round fits the occupancy the tile was sized for
// (2 workgroups per CU, 1 for the c = 128 64-row tile); ENCDIFF_ST_BWD_MF=0: the VALU form, A/B
template <int C, int R>
bool tail_bwd_mf(int nctx) {
  static const bool on = [] {
    const char* e = getenv("ENCDIFF_ST_BWD_MF");
    return !e || atoi(e) != 0;
  }();
  const size_t cap = (C == 128 && R == 64) ? 160 * 1024 : 80 * 1024;
  return on && TailBwd<C, R>::lds_bytes(nctx, true) <= cap;
}

template <int C, int R, bool MF>
int launch_tail_bwd_mf(const EncdiffStTailBwdArgs& p, hipStream_t s) {
  using T = TailBwd<C, R>;
  const size_t lds = T::lds_bytes(p.n_ctx, MF);
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)st_tail_bwd_kernel<C, R, MF>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr_ok != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)attr_ok;
  hipLaunchKernelGGL((st_tail_bwd_kernel<C, R, MF>), dim3((unsigned)(p.rows / R)), dim3(256), lds, s, p);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

template <int C, int R>
int launch_tail_bwd(const EncdiffStTailBwdArgs& p, hipStream_t s) {
  if (p.tokens % R || p.rows % R) return ENCDIFF_ERR_SHAPE;
  if (p.rows / R > p.part_rows) return ENCDIFF_ERR_SHAPE;
  if (p.tokens / R > 1 && (!p.kv_part || ((uintptr_t)p.kv_part & 15))) return ENCDIFF_ERR_ARG;
  if ((long)(p.rows / R) * p.n_ctx * 2 * C * 4 >= 0x7FFFFFF0L) return ENCDIFF_ERR_SHAPE;
  return tail_bwd_mf<C, R>(p.n_ctx) ? launch_tail_bwd_mf<C, R, true>(p, s) : launch_tail_bwd_mf<C, R, false>(p, s);
}

// ---------------------------------------------------------------------------------------------
template <int C, int R>
struct HeadBwd {
  static constexpr int LDT = C + 4, LDX = C + 8, LDQ = 3 * C + 8;
  static constexpr size_t ubytes() {
    const size_t a = (size_t)R * LDQ * 2, b = (size_t)R * LDT * 4;
    return ((a > b ? a : b) + 15) / 16 * 16;
  }
  static constexpr size_t lds_bytes() { return (size_t)R * LDT * 4 + 2 * (size_t)R * LDX * 2 + ubytes(); }
};

template <int C, int R>
__global__ __launch_bounds__(256) void st_head_bwd_kernel(const EncdiffStHeadBwdArgs p) {
  using T = HeadBwd<C, R>;
  constexpr int NWV = 4, NTH = 256, NT = C / (16 * NWV), LDT = T::LDT, LDX = T::LDX, LDQ = T::LDQ;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  float* Tr = (float*)smem_raw;
  bf16_t* Xa = (bf16_t*)(Tr + R * LDT);
  bf16_t* Xb = Xa + R * LDX;
  unsigned char* U = (unsigned char*)(Xb + R * LDX);
  bf16_t* Xq = (bf16_t*)U;  // [R][LDQ] d_qkv rows
  float* S = (float*)U;     // [R][LDT] LN1 terms (after the d_n1 GEMM)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row0 = blockIdx.x * R;
  const int n0 = wave * (C / NWV);
  if (p.kv_part) {
    // the tail kernel's dK2 | dV2 partial slabs of each image, summed in tile order (this grid's
    // workgroups share the (image, key, 4-channel) items)
    constexpr int C4 = 2 * C / 4;
    const int items = p.batch * p.n_ctx * C4;
    for (int e = blockIdx.x * NTH + tid; e < items; e += gridDim.x * NTH) {
      const int c4 = (e % C4) * 4, ij = e / C4, img = ij / p.n_ctx, j = ij - img * p.n_ctx;
      const float* src = p.kv_part + ((long)img * p.kv_tiles * p.n_ctx + j) * 2 * C + c4;
      float4 a = *(const float4*)src;
      for (int z = 1; z < p.kv_tiles; ++z) {
        const float4 v = *(const float4*)(src + (long)z * p.n_ctx * 2 * C);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
      bf16_t* dst = c4 < C ? (bf16_t*)p.dk2 + (long)ij * p.ld_dkv + c4 : (bf16_t*)p.dv2 + (long)ij * p.ld_dkv + (c4 - C);
      *(uint2*)dst = make_uint2(pack2(a.x, a.y), pack2(a.z, a.w));
    }
  }
  BFrags<NT, 3 * C> wqkv;
  BFrags<NT, C> win;
  load_b(wqkv, (const bf16_t*)p.w_qkv_t, 3 * C, n0, 0, lane);
  load_b(win, (const bf16_t*)p.w_in_t, C, n0, 0, lane);
  LnIn<C, R, NTH> ln1;  // t0 rows + LN1 statistics, in flight during the staging and the d_n1 GEMM
  ln_load<C, R, NTH>(ln1, (const bf16_t*)p.t0 + (long)row0 * p.ld_t0, p.ld_t0, p.s1 + 2L * row0, tid);
  rows_to_lds<3 * C, R, NTH>(Xq, LDQ, (const bf16_t*)p.d_qkv + (long)row0 * p.ld_dqkv, p.ld_dqkv, tid);
  {
    constexpr int CH = C / 8;
    const bf16_t* g = (const bf16_t*)p.d_t1 + (long)row0 * p.ld_dt1;
    for (int e = tid; e < R * CH; e += NTH) {
      const int r = e / CH, c8 = (e - r * CH) * 8;
      float f[8];
      unpack8(*(const uint4*)(g + (long)r * p.ld_dt1 + c8), f);
      *(float4*)(Tr + r * LDT + c8) = make_float4(f[0], f[1], f[2], f[3]);
      *(float4*)(Tr + r * LDT + c8 + 4) = make_float4(f[4], f[5], f[6], f[7]);
    }
  }
  __syncthreads();
  v4f acc[R / 16][NT];
  // ---- d_n1 = d_qkv Wqkv -> Xa (bf16)
  zero(acc);
  mma(acc, Xq, LDQ, wqkv, lane);
  acc_store_bf(acc, Xa, LDX, n0, lane);
  __syncthreads();
  // ---- d_t0 = d_t1 + LN1'(t0; d_n1)
  ln_bwd_rows<C, R, NTH>(Tr, LDT, Xa, LDX, Xb, ln1, p.g1, S, tid);
  __syncthreads();
  ln_partials<C, R>(S, LDT, Xa, LDX, p.ln1_dg, p.ln1_db, blockIdx.x, p.ld_part, tid);
  rows_to_global<C, R, NTH>((bf16_t*)p.d_t0 + (long)row0 * p.ld_dt0, p.ld_dt0, Xb, LDX, tid);
  // ---- d_gn = d_t0 Win
  zero(acc);
  mma(acc, Xb, LDX, win, lane);
  __syncthreads();
  acc_store_bf(acc, Xa, LDX, n0, lane);
  __syncthreads();
  rows_to_global<C, R, NTH>((bf16_t*)p.d_gn + (long)row0 * p.ld_dgn, p.ld_dgn, Xa, LDX, tid);
}

template <int C, int R>
int launch_head_bwd(const EncdiffStHeadBwdArgs& p, hipStream_t s) {
  using T = HeadBwd<C, R>;
  if (p.rows % R) return ENCDIFF_ERR_SHAPE;
  if (p.rows / R > p.part_rows) return ENCDIFF_ERR_SHAPE;
  constexpr size_t lds = T::lds_bytes();
  static_assert(lds <= 160 * 1024, "head backward LDS");
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)st_head_bwd_kernel<C, R>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr_ok != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)attr_ok;
  hipLaunchKernelGGL((st_head_bwd_kernel<C, R>), dim3((unsigned)(p.rows / R)), dim3(256), lds, s, p);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

// ---------------------------------------------------------------------------------------------
// The block's weight gradients dW += dY^T X (+ db += column sums of dY) over the tokens K, for the
// Linear layers of a fused transformer backward, as ONE grid: a workgroup owns a BM x BN output block
// (BM = 64 WM, BN = 16 WN; large enough that each operand is read about once per block row /
// column -- the 64 x 64 parts of the generic grouped launch re-read n3 eight times for ff.net.0.proj)
// over a chunk of kc tokens.  Stages of 32 tokens of dY [32][BM] and X [32][BN] are staged in LDS
// row-major (16-byte loads one stage ahead in registers, double-buffered LDS) and both operands are
// read k-outer with the gfx950 transpose read ds_read_b64_tr_b16; the 4 waves split BM.  Chunks
// write fp32 slabs that st_wgrad_fold_kernel sums in chunk order (reproducible); a single-chunk
// block accumulates straight into dW.
// (WM, WN) kinds: 16-row tiles per wave x 16-column tiles (acc WM * WN * 4 VGPRs <= 128)
constexpr int STWG_KINDS[][2] = {{1, 4}, {1, 16}, {4, 4}, {3, 4}, {2, 8}, {2, 16}, {4, 8}, {3, 8}};

#ifndef STWG_PF
#define STWG_PF 1
#endif
#ifndef ED_HEADBWD64_R32
#define ED_HEADBWD64_R32 0  // A/B: the c = 64 head backward on 32-row tiles at training batches too
#endif
#ifndef STWG_PF_TILES
#define STWG_PF_TILES 16
#endif
template <int WM, int WN>
struct WgShape {
  static constexpr int BM = 64 * WM, BN = 16 * WN, LDA = BM + 8, LDB = BN + 8;
  static constexpr int STAGE = 32 * (LDA + LDB);      // bf16 elements per stage
  static constexpr int NL = (BM + BN) / 64;           // 16-byte loads per thread per stage
  static constexpr size_t LDS = 2 * (size_t)STAGE * 2 + 16 * 4 * WM * 4;  // + bias reduction
  static constexpr int PF = WM * WN <= STWG_PF_TILES ? STWG_PF : 1;    // stages in flight (registers)
};

template <int WM, int WN>
__device__ __forceinline__ void st_wgrad_body(const StWg& p, int mblk, int nblk, int z, unsigned char* smem) {
  using T = WgShape<WM, WN>;
  constexpr int BM = T::BM, BN = T::BN, LDA = T::LDA, LDB = T::LDB, NL = T::NL;
  bf16_t* buf = (bf16_t*)smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, l16 = lane & 15, g4 = lane >> 4;
  const int tq = l16 >> 2, tp = l16 & 3;
  const int m0 = mblk * BM, n0 = nblk * BN;
  const int k0 = z * p.kc, k1 = min(p.K, k0 + p.kc), ns = (k1 - k0) / 32;
  const bool bias = p.db && nblk == 0;
  // stage loader: chunk e of the stage (row, 8-column piece) -- dY pieces first, then X
  auto load = [&](v4u32 (&r)[NL], int s) {
    const int k = k0 + 32 * s;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int e = tid + 256 * u;
      if (e < 4 * BM) {
        const int row = e / (BM / 8), c8 = (e % (BM / 8)) * 8;
        r[u] = *(const v4u32*)(p.dy + (long)(k + row) * p.ld_dy + m0 + c8);
      } else {
        const int f = e - 4 * BM, row = f / (BN / 8), c8 = (f % (BN / 8)) * 8;
        r[u] = *(const v4u32*)(p.x + (long)(k + row) * p.ld_x + n0 + c8);
      }
    }
  };
  auto store = [&](const v4u32 (&r)[NL], int b) {
    bf16_t* A = buf + b * T::STAGE;
    bf16_t* Bt = A + 32 * LDA;
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int e = tid + 256 * u;
      if (e < 4 * BM) {
        const int row = e / (BM / 8), c8 = (e % (BM / 8)) * 8;
        *(v4u32*)(A + row * LDA + c8) = r[u];
      } else {
        const int f = e - 4 * BM, row = f / (BN / 8), c8 = (f % (BN / 8)) * 8;
        *(v4u32*)(Bt + row * LDB + c8) = r[u];
      }
    }
  };
  // k-outer fragment of column col: k = g4 * 8 .. +8 (two transposed 4 x 16 reads)
  typedef __attribute__((address_space(3))) v4s lds_v4s;
  auto frag = [&](const bf16_t* tile, int ld, int col) -> v8bf {
    const bf16_t* a0 = tile + (g4 * 8 + tq) * ld + col + 4 * tp;
    const v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0));
    const v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(a0 + 4 * ld));
    const v8s r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8bf, r);
  };
  v4f acc[WM][WN];
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  float bs[WM];
#pragma unroll
  for (int i = 0; i < WM; ++i) bs[i] = 0.f;
  // register ring of PF stages in flight (PF - 1 stage loads outstanding while a stage is stored
  // to LDS): a stage is one global-load round trip, the kernel's critical path
  constexpr int PF = T::PF;
  v4u32 r[PF][NL];
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < ns) load(r[u], u);
  store(r[0], 0);
  __syncthreads();
  const int wm0 = wave * 16 * WM;  // this wave's rows of the block
  for (int s0 = 0; s0 < ns; s0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int s = s0 + u;
      if (s >= ns) break;
      if (s + PF < ns) load(r[u], s + PF);  // r[u]'s stage s is already in LDS
      const bf16_t* A = buf + (s & 1) * T::STAGE;
      const bf16_t* Bt = A + 32 * LDA;
      v8bf af[WM], bf[WN];
#pragma unroll
      for (int i = 0; i < WM; ++i) af[i] = frag(A, LDA, wm0 + 16 * i);
#pragma unroll
      for (int j = 0; j < WN; ++j) bf[j] = frag(Bt, LDB, 16 * j);
#pragma unroll
      for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[j], acc[i][j], 0, 0, 0);
      if (bias) {
#pragma unroll
        for (int i = 0; i < WM; ++i) {
          const v8s a = __builtin_bit_cast(v8s, af[i]);
          float t = 0.f;
#pragma unroll
          for (int e = 0; e < 8; ++e) t += bf2f((bf16_t)a[e]);
          bs[i] += t;
        }
      }
      if (s + 1 < ns) store(r[(u + 1) % PF], (s + 1) & 1);
      __syncthreads();
    }
  }
  // accumulator (i, j, q): row wm0 + 16 i + 4 g4 + q of the block, column 16 j + l16
  const bool direct = p.kb == 1;
  float* out = direct ? p.dw : p.slab + (long)z * p.M * p.N;
  const long ldo = direct ? p.ld_dw : p.N;
#pragma unroll
  for (int i = 0; i < WM; ++i)
#pragma unroll
    for (int j = 0; j < WN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float* o = out + (long)(m0 + wm0 + 16 * i + 4 * g4 + q) * ldo + n0 + 16 * j + l16;
        *o = direct ? *o + acc[i][j][q] : acc[i][j][q];
      }
  if (bias) {  // column sums of this chunk's dY: lane (l16, g4) holds 8 rows' sum -> add the 4 g4 groups
#pragma unroll
    for (int i = 0; i < WM; ++i) {
      float t = bs[i];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      if (g4 == 0) {
        const int m = m0 + wm0 + 16 * i + l16;
        if (direct) p.db[m] += t;
        else p.slab[(long)p.kb * p.M * p.N + (long)z * p.M + m] = t;
      }
    }
  }
}

template <int K>
__device__ __forceinline__ void st_wgrad_dispatch(const StWg& p, int mb, int nb, int z, unsigned char* smem) {
  if constexpr (K < (int)(sizeof(STWG_KINDS) / sizeof(STWG_KINDS[0]))) {
    if (p.kind == K) {
      st_wgrad_body<STWG_KINDS[K][0], STWG_KINDS[K][1]>(p, mb, nb, z, smem);
      return;
    }
    st_wgrad_dispatch<K + 1>(p, mb, nb, z, smem);
  }
}

__global__ __launch_bounds__(256, 2) void st_wgrad_kernel(const StWg* __restrict__ probs, int nprob) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  int pi = 0;
  for (int q = 1; q < nprob; ++q)
    if ((int)blockIdx.x >= probs[q].item0) pi = q;
  const StWg p = probs[pi];
  const int loc = blockIdx.x - p.item0;
  const int z = loc % p.kb, blk = loc / p.kb;  // a block's chunks adjacent: one XCD round-robin apart
  st_wgrad_dispatch<0>(p, blk % p.mb, blk / p.mb, z, smem_raw);
}

// the fold as its own launch (encdiff_st_wgrad_launch); encdiff_st_wgrad_launch_nofold leaves it to
// the next GroupNorm backward, whose grid carries the same blocks (norm.hip, stwg_fold_block)
__global__ __launch_bounds__(256) void st_wgrad_fold_kernel(const StWg* __restrict__ probs, int nprob) {
  __shared__ float4 red[8][32];
  stwg_fold_block(probs, nprob, blockIdx.x, red);
}

size_t stwg_lds(int kind) {
  switch (kind) {
    case 0: return WgShape<1, 4>::LDS;
    case 1: return WgShape<1, 16>::LDS;
    case 2: return WgShape<4, 4>::LDS;
    case 3: return WgShape<3, 4>::LDS;
    case 4: return WgShape<2, 8>::LDS;
    case 5: return WgShape<2, 16>::LDS;
    case 6: return WgShape<4, 8>::LDS;
    default: return WgShape<3, 8>::LDS;
  }
}

bool a16(const void* q) { return q && ((uintptr_t)q & 15) == 0; }

}  // namespace

extern "C" int encdiff_st_tail_bwd(const EncdiffStTailBwdArgs* a, void* stream) {
  if (!a) return ENCDIFF_ERR_ARG;
  const EncdiffStTailBwdArgs& p = *a;
  if (p.heads != 8 || (p.c != 64 && p.c != 128)) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.n_ctx < 1 || p.n_ctx > 64 || p.tokens < 1 || p.rows < 1 || p.rows % p.tokens || p.part_rows < 1)
    return ENCDIFF_ERR_SHAPE;
  const void* ptrs[] = {p.dy, p.f, p.t2, p.t1, p.q2, p.o2, p.k2, p.v2, p.w_po_t, p.w_ff2_t, p.w_ff1_t,
                        p.w_out2_t, p.w_q2_t, p.w_out1_t, p.d_t3, p.d_t2, p.d_q2, p.d_t1, p.d_o1, p.d_f, p.dk2, p.dv2};
  for (const void* q : ptrs)
    if (!a16(q)) return ENCDIFF_ERR_ARG;
  const long lds[] = {p.ld_dy, p.ld_f, p.ld_save, p.ld_kv, p.ld_d, p.ld_df, p.ld_dkv};
  for (long l : lds)
    if (l % 8) return ENCDIFF_ERR_ARG;
  if (!p.s3 || !p.s2 || !p.lse2 || !p.g3 || !p.g2 || !p.ln3_dg || !p.ln3_db || !p.ln2_dg || !p.ln2_db || p.ld_part < p.c)
    return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  switch (encdiff_st_tail_bwd_tile(p.c, p.rows, p.tokens)) {
    case 64: return p.c == 64 ? launch_tail_bwd<64, 64>(p, s) : launch_tail_bwd<128, 64>(p, s);
    default: return launch_tail_bwd<128, 32>(p, s);
  }
}

// c = 64: 64-row tiles; c = 128: 64-row tiles (116 KiB of LDS, one workgroup per CU) when they fill
// the chip, else 32 (two per CU)
extern "C" int encdiff_st_tail_bwd_tile(int c, int rows, int tokens) {
  if (c == 64) return 64;
  return rows / 64 >= 256 && tokens % 64 == 0 ? 64 : 32;
}

extern "C" int encdiff_st_head_bwd(const EncdiffStHeadBwdArgs* a, void* stream) {
  if (!a) return ENCDIFF_ERR_ARG;
  const EncdiffStHeadBwdArgs& p = *a;
  if (p.c != 64 && p.c != 128) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.rows < 1 || p.part_rows < 1) return ENCDIFF_ERR_SHAPE;
  const void* ptrs[] = {p.d_qkv, p.d_t1, p.t0, p.w_qkv_t, p.w_in_t, p.d_t0, p.d_gn};
  for (const void* q : ptrs)
    if (!a16(q)) return ENCDIFF_ERR_ARG;
  const long lds[] = {p.ld_dqkv, p.ld_dt1, p.ld_t0, p.ld_dt0, p.ld_dgn};
  for (long l : lds)
    if (l % 8) return ENCDIFF_ERR_ARG;
  if (!p.s1 || !p.g1 || !p.ln1_dg || !p.ln1_db || p.ld_part < p.c) return ENCDIFF_ERR_ARG;
  if (p.kv_part && (((uintptr_t)p.kv_part & 15) || p.kv_tiles < 1 || p.n_ctx < 1 || p.batch < 1 || !p.dk2 || !p.dv2 ||
                    ((uintptr_t)p.dk2 & 7) || ((uintptr_t)p.dv2 & 7) || p.ld_dkv % 4))
    return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (p.c == 64)
    return !ED_HEADBWD64_R32 && p.rows % 64 == 0 && p.rows / 64 >= 256 ? launch_head_bwd<64, 64>(p, s)
                                                                        : launch_head_bwd<64, 32>(p, s);
  return launch_head_bwd<128, 32>(p, s);
}

// Plan of encdiff_st_wgrad_launch: per problem the block shape (BM: the largest of 256 / 192 / 128 /
// 64 dividing M; BN: the largest of 256 / 128 / 64 dividing N with at most 32 accumulator tiles per
// wave), the token chunk (about 2 workgroups per CU over the whole group, >= 128 tokens, <= 64 chunks
// per block) and the fp32 slab region of the caller's workspace.
extern "C" int encdiff_st_wgrad_plan(const EncdiffWgradProb* in, int n, float* ws, long ws_floats, void* blob,
                                     long capacity, long* blob_bytes) {
  if (!in || n < 1 || n > STWG_MAXP || !blob_bytes || ws_floats < 0) return ENCDIFF_ERR_ARG;
  StWg w[STWG_MAXP];
  // tokens per chunk: a block's chunk is a chain of 32-token stages, each about one global-load round
  // trip (one stage prefetched), so chunks are cut by length, not by flops (ENCDIFF_STWG_KC; in the
  // step 256 -> 8.923, 512 -> 8.937, 1024 -> 9.045 ms, the generic grouped launch 8.971); doubled
  // until the chunks' slabs fit the workspace (large batches)
  static const int kc_env = [] {
    const char* e = getenv("ENCDIFF_STWG_KC");
    return e ? atoi(e) : 256;
  }();
  int items = 0, folds = 0;
  for (long kc0 = (kc_env + 31) / 32 * 32;; kc0 *= 2) {
    long ws_used = 0;
    bool fits = true;
    items = folds = 0;
    for (int i = 0; i < n; ++i) {
      const EncdiffWgradProb& q = in[i];
      if (!q.dy || !q.x || !q.dw || ((uintptr_t)q.dy & 15) || ((uintptr_t)q.x & 15) || q.ld_dy % 8 || q.ld_x % 8)
        return ENCDIFF_ERR_ARG;
      if (q.M % 64 || q.N % 64 || q.K % 32 || q.K <= 0 || q.ld_dw < q.N) return ENCDIFF_ERR_SHAPE;
      StWg& p = w[i];
      p.dy = (const bf16_t*)q.dy; p.x = (const bf16_t*)q.x; p.dw = q.dw; p.db = q.db;
      p.ld_dy = q.ld_dy; p.ld_x = q.ld_x; p.ld_dw = q.ld_dw;
      p.M = q.M; p.N = q.N; p.K = q.K;
      int bm = 64;
      for (int c : {256, 192, 128})
        if (q.M % c == 0) { bm = c; break; }
      const int wm = bm / 64;
      int bn = 64;
      for (int c : {256, 128})
        if (q.N % c == 0 && wm * (c / 16) <= 32) { bn = c; break; }
      int kind = -1;
      for (int k = 0; k < (int)(sizeof(STWG_KINDS) / sizeof(STWG_KINDS[0])); ++k)
        if (STWG_KINDS[k][0] == wm && STWG_KINDS[k][1] == bn / 16) kind = k;
      if (kind < 0) return ENCDIFF_ERR_UNSUPPORTED;
      p.kind = kind; p.bm = bm; p.bn = bn;
      p.mb = q.M / bm; p.nb = q.N / bn;
      long kc = kc0 < 32 ? 32 : kc0;
      if (kc > q.K) kc = q.K;
      const long kb = (q.K + kc - 1) / kc;
      p.kc = (int)kc; p.kb = (int)kb;
      p.slab = nullptr;
      if (kb > 1) {
        const long need = ((long)kb * q.M * q.N + (q.db ? (long)kb * q.M : 0) + 31) & ~31L;
        if (!ws || ws_used + need > ws_floats) {
          fits = false;
          break;
        }
        p.slab = ws + ws_used;
        ws_used += need;
      }
      p.item0 = items;
      items += p.mb * p.nb * (int)kb;
      p.fold0 = folds;
      if (kb > 1) folds += (int)(((long)q.M * q.N / 4 + 31) / 32 + (q.db ? (q.M + 31) / 32 : 0));
    }
    if (fits) break;
    if (kc0 >= (1L << 30)) return ENCDIFF_ERR_SHAPE;
  }
  const long probs_off = 64;
  const long bytes = probs_off + (long)sizeof(StWg) * n;
  *blob_bytes = bytes;
  if (!blob) return ENCDIFF_OK;
  if (capacity < bytes || ((uintptr_t)blob & 7)) return ENCDIFF_ERR_ARG;
  StWgHead h{STWG_MAGIC, n, items, folds, probs_off, bytes};
  char* out = (char*)blob;
  std::memset(out, 0, (size_t)bytes);
  std::memcpy(out, &h, sizeof(h));
  std::memcpy(out + probs_off, w, sizeof(StWg) * (size_t)n);
  return ENCDIFF_OK;
}

namespace {
int stwg_launch(const void* host_blob, const void* dev_blob, void* stream, bool fold, int* nfold) {
  if (!host_blob || !dev_blob) return ENCDIFF_ERR_ARG;
  StWgHead h;
  std::memcpy(&h, host_blob, sizeof(h));
  if (h.magic != STWG_MAGIC || h.nprob < 1 || h.nprob > STWG_MAXP || h.nitems < 1) return ENCDIFF_ERR_ARG;
  const StWg* hp = (const StWg*)((const char*)host_blob + h.probs_off);
  size_t lds = 0;
  for (int i = 0; i < h.nprob; ++i) lds = std::max(lds, stwg_lds(hp[i].kind));
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)st_wgrad_kernel,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (attr_ok != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)attr_ok;
  const StWg* dp = (const StWg*)((const char*)dev_blob + h.probs_off);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(st_wgrad_kernel, dim3((unsigned)h.nitems), dim3(256), lds, s, dp, h.nprob);
  if (fold && h.nfold > 0) hipLaunchKernelGGL(st_wgrad_fold_kernel, dim3((unsigned)h.nfold), dim3(256), 0, s, dp, h.nprob);
  if (nfold) *nfold = h.nfold;
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}
}  // namespace

extern "C" int encdiff_st_wgrad_launch(const void* host_blob, const void* dev_blob, void* stream) {
  return stwg_launch(host_blob, dev_blob, stream, true, nullptr);
}

extern "C" int encdiff_st_wgrad_launch_nofold(const void* host_blob, const void* dev_blob, void* stream,
                                              const void** fold_plan, int* fold_blocks) {
  if (!fold_plan || !fold_blocks) return ENCDIFF_ERR_ARG;
  const int rc = stwg_launch(host_blob, dev_blob, stream, false, fold_blocks);
  *fold_plan = rc == ENCDIFF_OK && *fold_blocks > 0 ? dev_blob : nullptr;
  if (rc != ENCDIFF_OK || !*fold_plan) *fold_blocks = 0;
  return rc;
}
