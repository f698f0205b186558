// norm.hip -- GroupNorm(+FiLM)(+SiLU) and LayerNorm, forward and backward, NHWC bf16.
//
// GroupNorm: one workgroup per (image, slice of whole groups); the slice is held in
// registers between the statistics (fp32, two-pass, as GroupNorm32 computes in fp32:
// util.py:242-244) and the write of the normalised, FiLM-modulated, SiLU-activated
// output (openaimodel_enc.py:201-205, 225-232, 267-271, 684-686; attention.py:76-77).
// The backward recomputes the forward from x and the saved statistics and emits
// per-image partial sums for dgamma/dbeta (reduced once per step by
// encdiff_reduce_partials) and the FiLM gradients d(scale), d(shift) per (b, c).
#include <stdlib.h>

#include "common.h"
#include "stwg.h"

namespace {

#ifndef ED_GN_STAMP
#define ED_GN_STAMP 0  // diagnostic builds: phase stamps of the GroupNorm backward (tools/gn_stamps.py)
#endif
#ifndef ED_GN_SLAB_U
#define ED_GN_SLAB_U 1  // backward, dy from slabs: rows per load batch
#endif
#ifndef ED_LN_BWD_U
#define ED_LN_BWD_U 2  // LayerNorm backward rows per thread in flight (4 measured slower: 9.09 -> 9.11 ms/step)
#endif
#ifndef GN_BWD_LDS_FULL
#define GN_BWD_LDS_FULL 0
#endif
#ifndef ED_GN_BWD_U
#define ED_GN_BWD_U 4  // backward rows per load batch (code size vs loads in flight)
#endif
constexpr int GN_THREADS = 256;
constexpr int GN_TILE = 1024;      // backward: 16-byte vectors of a slice kept in LDS per operand (16 KB)
constexpr int GN_TILE_FWD = 6144;  // forward: dynamic LDS tile up to 96 KB (the VQ encoder's 64x64 levels)

// A workgroup owns (image b, channel slice [c0, c0 + cs)); cs is a multiple of 8 and of
// channels-per-group, so every group lies inside one slice and the slices are independent.
// Threads: tv = channel vector (8 channels) of the slice, tp = pixel lane.  The slice is
// read from HBM once into an LDS tile (slices larger than GN_TILE vectors re-read HBM/L2),
// per-channel partials are reduced deterministically (wave shuffles + ordered LDS sums),
// statistics are two-pass (mean, then centred sum of squares).  Loops stay rolled (4-way
// unrolled) so the kernels are a few hundred instructions: a cold instruction cache is
// otherwise the dominant latency of these small launches.
// Workgroup -> (image, slice) index, XCD-aware: workgroup i runs on XCD i % 8, and the slices of
// one image share every 128-B line of its rows (a slice is a channel range), so consecutive
// slice indices go to consecutive workgroups OF ONE XCD -- each line is fetched into one L2.
// Bijective when the grid is a multiple of 8 (else identity).
ED_DEV int gn_xcd_index(int i, int n) { return (n & 7) ? i : (i & 7) * (n >> 3) + (i >> 3); }

struct GnSlice {
  int S, b, c0, cs, nvc, np, tv, tp, cpg, gs, g0, cb;
  bool active, tiled;
  ED_DEV GnSlice(const EncdiffGroupNormArgs& p, int cs_, int tile_cap = GN_TILE, int nblk = 0) {
    cs = cs_;
    S = p.c / cs;
    const int bid = gn_xcd_index(blockIdx.x, nblk ? nblk : gridDim.x);
    b = bid / S;
    c0 = (bid - b * S) * cs;
    nvc = cs >> 3;
    np = GN_THREADS / nvc;
    tv = threadIdx.x % nvc;
    tp = threadIdx.x / nvc;
    active = tp < np;
    cpg = p.c / p.groups;
    gs = cs / cpg;
    g0 = c0 / cpg;
    cb = c0 + tv * 8;
    tiled = nvc * p.hw <= tile_cap;
  }
};

ED_DEV void load8f(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// Deterministic reduction of per-thread channel partials q[NQ][8] over the pixel lanes of
// the slice into out[NQ][cs] (LDS).  Power-of-two nvc: xor-shuffles inside each wave, then
// the wave rows are added in order; otherwise every pixel-lane row goes through LDS and a
// thread per channel adds the rows in order.  Ends with a barrier.
// First half of slice_reduce: the per-lane partials reduced across lanes into `rows` partial rows
// red[(r * NQ + k) * cs + c] (ends with a barrier); returns rows.
template <int NQ>
ED_DEV int slice_partials(float (&q)[NQ][8], const GnSlice& L, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool pow2 = (L.nvc & (L.nvc - 1)) == 0;
  int rows;
  if (pow2) {
    // Butterfly reduce-scatter over the lanes sharing tv (lane bits >= log2(nvc)): at each of
    // the first three levels a lane keeps half of its channel set and sends the other half
    // (4, 2, 1 shuffles per k instead of 8), so after them it owns ONE channel's partial;
    // further levels add single values.  ~9 shuffles per k instead of 40 (nvc = 2): the
    // shuffles (ds_bpermute, LDS latency each) were the latency chain of the whole kernel.
    int c = 0, hs = 4, off = L.nvc;
#pragma unroll
    for (int lvl = 0; lvl < 3; ++lvl, hs >>= 1) {
      if (off < 64) {
        const bool hi = (lane & off) != 0;
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
          float send[4], recv[4];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < hs) send[i] = hi ? q[k][i] : q[k][i + hs];
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < hs) recv[i] = __shfl_xor(send[i], off, 64);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (i < hs) q[k][i] = (hi ? q[k][i + hs] : q[k][i]) + recv[i];
        }
        c += hi ? hs : 0;
        off <<= 1;
      }
    }
    const int nval = 8 >> __builtin_ctz((unsigned)(off / L.nvc));  // 8 >> (butterfly levels done)
    for (; off < 64; off <<= 1) {
#pragma unroll
      for (int k = 0; k < NQ; ++k) q[k][0] += __shfl_xor(q[k][0], off, 64);
    }
    // lanes whose remaining-level bits are zero hold the totals of channels c .. c+nval-1
    // (nval = 1 after three butterfly levels; 2, 4, 8 when fewer levels exist)
    const int owner_mask = 63 & ~(L.nvc * 8 - 1);
    if ((lane & owner_mask) == 0) {
#pragma unroll
      for (int k = 0; k < NQ; ++k)
        for (int i = 0; i < nval; ++i) red[(wave * NQ + k) * L.cs + L.tv * 8 + c + i] = q[k][i];
    }
    rows = L.nvc >= 64 ? GN_THREADS / L.nvc : GN_THREADS / 64;
  } else {
    if (L.active) {
#pragma unroll
      for (int k = 0; k < NQ; ++k)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[(L.tp * NQ + k) * L.cs + L.tv * 8 + i] = q[k][i];
    }
    rows = L.np;
  }
  __syncthreads();
  return rows;
}

template <int NQ>
ED_DEV void slice_reduce(float (&q)[NQ][8], const GnSlice& L, float* red, float* out) {
  const int rows = slice_partials<NQ>(q, L, red);
  for (int e = threadIdx.x; e < NQ * L.cs; e += GN_THREADS) {
    const int k = e / L.cs, c = e - k * L.cs;
    float a = 0.f;
    for (int r = 0; r < rows; ++r) a += red[(r * NQ + k) * L.cs + c];
    out[k * L.cs + c] = a;
  }
  __syncthreads();
}

// Row px of the thread's channel vector: from the LDS tile when the slice fits, else HBM/L2.
ED_DEV uint4 gn_row(const GnSlice& L, const uint4* tile, const bf16_t* g, long ld, int px) {
  return L.tiled ? tile[px * L.nvc + L.tv] : *(const uint4*)(g + (long)px * ld);
}

// x as the deferred split-K finalize of its producer GEMM (EncdiffGroupNormArgs.x_from): fp32
// slabs [split][M][C] behind ws, C = alpha * sum_z slab[z] (+ bias)(+ resid) -- gemm.hip's
// gemm_finalize, same summation order (one ordered sum up to 8 slabs, else four z-groups added
// ((0 + 1) + 2) + 3), same rounding -- so x is bitwise what the finalize pass would have written.
struct GnSlabs {
  const float* ws;  // NULL: x is read from memory
  long total;       // M * C
  int split;
  float alpha;
  const float* bias;
  const bf16_t* resid;
  long ld_resid;
};

// Slabs are loaded 8 at a time, every load of a batch issued before the first add (a chain of
// dependent loads per slab made the small-batch launches latency-bound: 32 slabs at B = 8).
ED_DEV void gn_slab_batch(const float* w, long stride, int z0, int split, float (&v)[8][8]) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (z0 + j < split) {
      load8f(w + (long)(z0 + j) * stride, v[j]);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[j][i] = 0.f;
    }
  }
}

ED_DEV uint4 gn_slab_row(const GnSlabs& sl, long row, int c, int cb) {
  // alpha / bias through splitk_scale: gemm.hip's gemm_finalize does this combine too, bitwise alike
  const float* w = sl.ws + row * c + cb;
  float a[8], v[8][8];
  if (sl.split <= 8) {
    gn_slab_batch(w, sl.total, 0, sl.split, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (j < sl.split) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] += v[j][i];
      }
    }
  } else {  // z-group k sums slabs k, k + 4, ... in order
    float g[4][8];
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) g[k][i] = 0.f;
    for (int z0 = 0; z0 < sl.split; z0 += 8) {
      gn_slab_batch(w, sl.total, z0, sl.split, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (z0 + j < sl.split) {
#pragma unroll
          for (int i = 0; i < 8; ++i) g[j & 3][i] += v[j][i];
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = ((g[0][i] + g[1][i]) + g[2][i]) + g[3][i];
  }
  float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (sl.bias) load8f(sl.bias + cb, bb);
#pragma unroll
  for (int i = 0; i < 8; ++i) a[i] = splitk_scale(a[i], sl.alpha, bb[i]);
  if (sl.resid) {
    float r[8];
    unpack8(*(const uint4*)(sl.resid + row * sl.ld_resid + cb), r);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += r[i];
  }
  return pack8(a);
}

// phase 0: stream the slice from HBM (4 loads in flight per thread), fill the tile, and
// accumulate the per-channel sum and sum of squares in the same pass.  With slabs, x is
// combined from them first and written back (the producer's output).
ED_DEV void gn_stream_in(const GnSlice& L, uint4* tile, const bf16_t* X, long ld, int HW, float* s, float* ss,
                         const GnSlabs& sl, int C) {
  auto acc = [&](const uint4& u, int px) {
    if (L.tiled) tile[px * L.nvc + L.tv] = u;
    float v[8];
    unpack8(u, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) { s[i] += v[i]; ss[i] += v[i] * v[i]; }
  };
  if (sl.ws) {  // (rolled: a row already has up to 8 slab loads in flight)
    for (int px = L.tp; px < HW; px += L.np) {
      const uint4 u = gn_slab_row(sl, (long)L.b * HW + px, C, L.cb);
      *(uint4*)(const_cast<bf16_t*>(X) + (long)px * ld) = u;
      acc(u, px);
    }
    return;
  }
#pragma unroll 4
  for (int px = L.tp; px < HW; px += L.np) acc(*(const uint4*)(X + (long)px * ld), px);
}

// One reduction round: sum and sum of squares together (var = E[x^2] - mean^2 in fp32 over
// bf16 inputs of O(1) magnitude; the second read of the slice and a second reduction with
// its barriers were the longest part of this latency-bound kernel).
__global__ __launch_bounds__(GN_THREADS) void gn_fwd_kernel(const EncdiffGroupNormArgs p, int cs, int tile_cap,
                                                            const GnSlabs sl) {
  extern __shared__ uint4 tile[];  // tile_cap vectors (0: untiled, re-read from L2/HBM)
  __shared__ float red[4096], chs[1024], gsh[2 * 64];
  const GnSlice L(p, cs, tile_cap);
  const int HW = p.hw;
  const float inv_n = 1.f / ((float)HW * L.cpg);
  const bf16_t* X = (const bf16_t*)p.x + (long)L.b * HW * p.ldx + L.cb;
  float s[2][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[0][i] = s[1][i] = 0.f;
  if (L.active) gn_stream_in(L, tile, X, p.ldx, HW, s[0], s[1], sl, p.c);
  // per-channel affine / FiLM constants (independent of the statistics)
  float ga[8], be[8], sc[8], sf[8];
  load8f(p.gamma + L.cb, ga);
  load8f(p.beta + L.cb, be);
  if (p.film) {
    load8f(p.film + (long)L.b * p.ld_film + L.cb, sc);
    load8f(p.film + (long)L.b * p.ld_film + p.c + L.cb, sf);
  }
  slice_reduce<2>(s, L, red, chs);
  if (threadIdx.x < L.gs) {
    float a = 0.f, q = 0.f;
    for (int c = threadIdx.x * L.cpg; c < (threadIdx.x + 1) * L.cpg; ++c) { a += chs[c]; q += chs[L.cs + c]; }
    const float mean = a * inv_n;
    const float var = fmaxf(q * inv_n - mean * mean, 0.f);
    const float rstd = rsqrtf(var + p.eps);
    gsh[threadIdx.x] = mean;
    gsh[64 + threadIdx.x] = rstd;
    const long gi = (long)L.b * p.groups + L.g0 + threadIdx.x;
    p.stats[2 * gi] = mean;
    p.stats[2 * gi + 1] = rstd;
  }
  __syncthreads();
  if (!L.active) return;
  float mean[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) mean[i] = gsh[(L.tv * 8 + i) / L.cpg];
  float mul[8], add[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float r = gsh[64 + (L.tv * 8 + i) / L.cpg];
    // y = ((x - m) r ga + be)(1 + sc) + sh
    float a = r * ga[i], bb = be[i] - mean[i] * a;
    if (p.film) {
      a *= (1.f + sc[i]);
      bb = bb * (1.f + sc[i]) + sf[i];
    }
    mul[i] = a; add[i] = bb;
  }
  bf16_t* Y = (bf16_t*)p.y + (long)L.b * HW * p.ldy + L.cb;
  const bool silu = p.silu;
  bf16_t* DS = silu && p.dsilu ? (bf16_t*)p.dsilu + (long)L.b * HW * p.ld_dsilu + L.cb : nullptr;
  if (DS) {  // training: silu'(z) for the backward too
#pragma unroll 2
    for (int px = L.tp; px < HW; px += L.np) {
      float v[8], g[8];
      unpack8(gn_row(L, tile, X, p.ldx, px), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = silu_and_grad(v[i] * mul[i] + add[i], g[i]);
      *(uint4*)(Y + (long)px * p.ldy) = pack8(v);
      *(uint4*)(DS + (long)px * p.ld_dsilu) = pack8(g);
    }
    return;
  }
#pragma unroll 2
  for (int px = L.tp; px < HW; px += L.np) {
    float v[8];
    unpack8(gn_row(L, tile, X, p.ldx, px), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float z = v[i] * mul[i] + add[i];
      v[i] = silu ? silu_f(z) : z;
    }
    *(uint4*)(Y + (long)px * p.ldy) = pack8(v);
  }
}

// Forward from the producer GEMM's per-64-row-segment channel sums (p.in_stats): no
// reduction pass and no LDS tile -- x is streamed once.  The first PF rows of each thread are
// loaded before the group statistics are formed, so their latency overlaps it.
__global__ __launch_bounds__(GN_THREADS) void gn_fwd_stats_kernel(const EncdiffGroupNormArgs p, int cs) {
  __shared__ float gsh[2 * 64];
  const GnSlice L(p, cs, 0);
  const int HW = p.hw, nseg = HW >> 6;
  const bf16_t* X = (const bf16_t*)p.x + (long)L.b * HW * p.ldx + L.cb;
  constexpr int PF = 4;
  uint4 pre[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) {
    const int px = L.tp + i * L.np;
    pre[i] = (L.active && px < HW) ? *(const uint4*)(X + (long)px * p.ldx) : (uint4){0u, 0u, 0u, 0u};
  }
  // the slice's segment sums in one round trip: [2][nseg][cs] into LDS (host: nseg*cs <= 2048)
  __shared__ float pst[2 * 2048];
  const int ns = nseg * L.cs;
  for (int e = threadIdx.x; e < 2 * ns; e += GN_THREADS) {
    const int k = e / ns, r = e - k * ns, sg = r / L.cs, c = r - sg * L.cs;
    pst[e] = p.in_stats[(2 * ((long)L.b * nseg + sg) + k) * p.ld_in_stats + L.c0 + c];
  }
  __syncthreads();
  if (threadIdx.x < L.gs) {
    const float inv_n = 1.f / ((float)HW * L.cpg);
    const int c0 = threadIdx.x * L.cpg;
    float a = 0.f, q = 0.f;
    for (int sg = 0; sg < nseg; ++sg)
      for (int c = 0; c < L.cpg; ++c) { a += pst[sg * L.cs + c0 + c]; q += pst[ns + sg * L.cs + c0 + c]; }
    const float mean = a * inv_n;
    const float var = fmaxf(q * inv_n - mean * mean, 0.f);
    const float rstd = rsqrtf(var + p.eps);
    gsh[threadIdx.x] = mean;
    gsh[64 + threadIdx.x] = rstd;
    const long gi = (long)L.b * p.groups + L.g0 + threadIdx.x;
    p.stats[2 * gi] = mean;
    p.stats[2 * gi + 1] = rstd;
  }
  float ga[8], be[8], sc[8], sf[8];
  load8f(p.gamma + L.cb, ga);
  load8f(p.beta + L.cb, be);
  if (p.film) {
    load8f(p.film + (long)L.b * p.ld_film + L.cb, sc);
    load8f(p.film + (long)L.b * p.ld_film + p.c + L.cb, sf);
  }
  __syncthreads();
  if (!L.active) return;
  float mul[8], add[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = (L.tv * 8 + i) / L.cpg;
    const float r = gsh[64 + g];
    float a = r * ga[i], bb = be[i] - gsh[g] * a;
    if (p.film) {
      a *= (1.f + sc[i]);
      bb = bb * (1.f + sc[i]) + sf[i];
    }
    mul[i] = a; add[i] = bb;
  }
  bf16_t* Y = (bf16_t*)p.y + (long)L.b * HW * p.ldy + L.cb;
  const bool silu = p.silu;
  bf16_t* DS = silu && p.dsilu ? (bf16_t*)p.dsilu + (long)L.b * HW * p.ld_dsilu + L.cb : nullptr;
  auto emit = [&](const uint4& u, int px) {
    float v[8];
    unpack8(u, v);
    if (DS) {  // training: silu'(z) for the backward too
      float g[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = silu_and_grad(v[i] * mul[i] + add[i], g[i]);
      *(uint4*)(DS + (long)px * p.ld_dsilu) = pack8(g);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float z = v[i] * mul[i] + add[i];
        v[i] = silu ? silu_f(z) : z;
      }
    }
    *(uint4*)(Y + (long)px * p.ldy) = pack8(v);
  };
#pragma unroll
  for (int i = 0; i < PF; ++i) {
    const int px = L.tp + i * L.np;
    if (px < HW) emit(pre[i], px);
  }
#pragma unroll 2
  for (int px = L.tp + PF * L.np; px < HW; px += L.np) emit(*(const uint4*)(X + (long)px * p.ldx), px);
}

// Large images (hw >= 1024, the VQ encoder's levels): per-image group statistics from the
// producer's segment sums in a small kernel (thread (channel, segment lane) sums every J-th
// segment, lanes added in order), then a streaming apply over (pixel chunk, image) blocks that
// span all channels -- coalesced rows instead of the narrow channel slices a per-(image,
// slice) reduction needs.
__global__ __launch_bounds__(GN_THREADS) void gn_group_stats_kernel(const EncdiffGroupNormArgs p) {
  __shared__ float part[2][GN_THREADS];
  __shared__ float chs[2][512];
  const int b = blockIdx.x, C = p.c, nseg = p.hw >> 6, cpg = C / p.groups;
  for (int c0 = 0; c0 < C; c0 += GN_THREADS) {  // channel chunks of <= 256
    const int cw = min(GN_THREADS, C - c0), J = GN_THREADS / cw;
    const int c = threadIdx.x % cw, j = threadIdx.x / cw;
    float a = 0.f, q = 0.f;
    if (j < J) {
#pragma unroll 8
      for (int sg = j; sg < nseg; sg += J) {
        const float* st = p.in_stats + 2 * ((long)b * nseg + sg) * p.ld_in_stats + c0 + c;
        a += st[0];
        q += st[p.ld_in_stats];
      }
    }
    part[0][threadIdx.x] = a;
    part[1][threadIdx.x] = q;
    __syncthreads();
    if (threadIdx.x < cw) {
      float s0 = 0.f, s1 = 0.f;
      for (int k = 0; k < J; ++k) { s0 += part[0][k * cw + threadIdx.x]; s1 += part[1][k * cw + threadIdx.x]; }
      chs[0][c0 + threadIdx.x] = s0;
      chs[1][c0 + threadIdx.x] = s1;
    }
    __syncthreads();
  }
  if (threadIdx.x < p.groups) {
    float a = 0.f, q = 0.f;
    for (int c = threadIdx.x * cpg; c < (threadIdx.x + 1) * cpg; ++c) { a += chs[0][c]; q += chs[1][c]; }
    const float inv_n = 1.f / ((float)p.hw * cpg);
    const float mean = a * inv_n;
    const float var = fmaxf(q * inv_n - mean * mean, 0.f);
    const long gi = (long)b * p.groups + threadIdx.x;
    p.stats[2 * gi] = mean;
    p.stats[2 * gi + 1] = rsqrtf(var + p.eps);
  }
}

// streaming apply: block (chunk of rows, image b), all C channels; thread = (row lane, vector)
__global__ __launch_bounds__(GN_THREADS) void gn_apply_kernel(const EncdiffGroupNormArgs p, int rows_per_block) {
  const int b = blockIdx.y, nvc = p.c >> 3, np = GN_THREADS / nvc;
  const int tv = threadIdx.x % nvc, tp = threadIdx.x / nvc;
  if (tp >= np) return;
  const int cb = tv * 8, cpg = p.c / p.groups;
  float ga[8], be[8], sc[8], sf[8], mul[8], add[8];
  load8f(p.gamma + cb, ga);
  load8f(p.beta + cb, be);
  if (p.film) {
    load8f(p.film + (long)b * p.ld_film + cb, sc);
    load8f(p.film + (long)b * p.ld_film + p.c + cb, sf);
  }
  const float* st = p.stats + (long)b * p.groups * 2;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = (cb + i) / cpg;
    float a = st[2 * g + 1] * ga[i], bb = be[i] - st[2 * g] * a;
    if (p.film) {
      a *= (1.f + sc[i]);
      bb = bb * (1.f + sc[i]) + sf[i];
    }
    mul[i] = a; add[i] = bb;
  }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(p.hw, r0 + rows_per_block);
  const bf16_t* X = (const bf16_t*)p.x + (long)b * p.hw * p.ldx + cb;
  bf16_t* Y = (bf16_t*)p.y + (long)b * p.hw * p.ldy + cb;
  const bool silu = p.silu;
  bf16_t* DS = silu && p.dsilu ? (bf16_t*)p.dsilu + (long)b * p.hw * p.ld_dsilu + cb : nullptr;
  if (DS) {  // training: silu'(z) for the backward too
#pragma unroll 4
    for (int px = r0 + tp; px < r1; px += np) {
      float v[8], g[8];
      unpack8(*(const uint4*)(X + (long)px * p.ldx), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = silu_and_grad(v[i] * mul[i] + add[i], g[i]);
      *(uint4*)(Y + (long)px * p.ldy) = pack8(v);
      *(uint4*)(DS + (long)px * p.ld_dsilu) = pack8(g);
    }
    return;
  }
#pragma unroll 4
  for (int px = r0 + tp; px < r1; px += np) {
    float v[8];
    unpack8(*(const uint4*)(X + (long)px * p.ldx), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float z = v[i] * mul[i] + add[i];
      v[i] = silu ? silu_f(z) : z;
    }
    *(uint4*)(Y + (long)px * p.ldy) = pack8(v);
  }
}

// SLAB: dy is combined from its producer's deferred split-K slabs (a separate instantiation: the
// slab combine unrolled into the plain kernel doubled its code and pushed it past 256 VGPRs)
#if ED_GN_STAMP
// phase stamps of the GroupNorm backward (diagnostic builds only, tools/gn_stamps.py): per block,
// thread 0: [0] realtime at entry, [1..6] shader clock at entry / after the constants / after pass
// 1 / after the reduction / after the group terms / at exit, [7] realtime at exit
__device__ unsigned long long gn_stamps[16384][8];
#define GN_STAMP(i)                                                                        \
  do {                                                                                     \
    if (threadIdx.x == 0 && blockIdx.x < 16384) gn_stamps[blockIdx.x][i] = __builtin_readcyclecounter(); \
  } while (0)
#define GN_STAMP_RT(i)                                                                     \
  do {                                                                                     \
    if (threadIdx.x == 0 && blockIdx.x < 16384) gn_stamps[blockIdx.x][i] = wall_clock64(); \
  } while (0)
#else
#define GN_STAMP(i) do {} while (0)
#define GN_STAMP_RT(i) do {} while (0)
#endif

// dy / resid given at the resolution of a resample that follows this GroupNorm (its output feeds a
// 2x avg-pool or nearest-up, EncdiffGroupNormArgs.dy_resample / resid_resample): the adjoint of
// that resample read on the fly -- DOWN2: 0.25 * the parent pixel; UP2: the sum of the 4 children
// (in the order of the elementwise adjoint kernel, so the result is bitwise its output)
ED_DEV void gn_resample_adj(const bf16_t* base, long ld, int mode, int W, int px, float (&v)[8]) {
  const int y = px / W, x = px - y * W;
  if (mode == ENCDIFF_RESAMPLE_DOWN2) {
    unpack8(*(const uint4*)(base + (long)((y >> 1) * (W >> 1) + (x >> 1)) * ld), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] *= 0.25f;
  } else {
    const long r0 = (long)(2 * y) * (2 * W) + 2 * x;
    float t[8];
    unpack8(*(const uint4*)(base + r0 * ld), v);
    unpack8(*(const uint4*)(base + (r0 + 1) * ld), t);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += t[i];
    unpack8(*(const uint4*)(base + (r0 + 2 * W) * ld), t);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += t[i];
    unpack8(*(const uint4*)(base + (r0 + 2 * W + 1) * ld), t);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] += t[i];
  }
}
// pixels per image of a tensor at the other side of resample `mode` from hw
ED_DEV int gn_rs_hw(int mode, int hw) { return mode == ENCDIFF_RESAMPLE_DOWN2 ? hw >> 2 : (mode ? hw << 2 : hw); }

// RS: the resampled-operand variant (dy and / or resid through gn_resample_adj); separate so the
// common instantiations keep their registers
// DSL: the SiLU gradient is read from the forward's dsilu rows instead of recomputed from z
// LDS is dynamic, sized per launch (gn_bwd_lds): the pixel tiles only where pass 2 reads them (not
// for register-cached single-batch slices), the reduction rows for the slice's channel count -- a
// few KB for most UNet calls instead of a static ~74 KB, so the launch packs more workgroups per
// CU (the weight-gradient fold riding in it included)
template <bool SLAB, bool RS = false, bool DSL = false>
__global__ __launch_bounds__(GN_THREADS) void gn_bwd_kernel(const EncdiffGroupNormArgs p, int cs, const GnSlabs sl,
                                                            int ntile, int nred) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gn_smem[];
  uint4* tx = (uint4*)gn_smem;   // [ntile] x rows of the slice (tiled pass 2)
  uint4* td = tx + ntile;        // [ntile] dy rows
  float* red = (float*)(td + ntile);  // [nred] reduction rows, then the group-term scratch
  float* chs = red + nred;            // [2][cs] channel totals
  float* gam_sh = chs + 2 * cs;       // [cs]
  // workgroups past the GroupNorm's: the weight-gradient fold riding in this launch
  const int gnb = p.batch * (p.c / cs);
  if ((int)blockIdx.x >= gnb) {
    stwg_fold_from_blob(p.fold_plan, blockIdx.x - gnb, (float4(*)[32])red);
    return;
  }
  GN_STAMP_RT(0);
  GN_STAMP(1);
  const GnSlice L(p, cs, ntile, gnb);
  const int HW = p.hw;
  const bool film = p.film != nullptr, silu = p.silu;
  const float inv_n = 1.f / ((float)HW * L.cpg);
  const long off = (long)L.b * HW;
  const bf16_t* X = (const bf16_t*)p.x + off * p.ldx + L.cb;
  const int dyrs = RS ? p.dy_resample : 0, rsrs = RS ? p.resid_resample : 0;
  const bf16_t* DY = (const bf16_t*)p.dy + (long)L.b * gn_rs_hw(dyrs, HW) * p.lddy + L.cb;
  // dy row px (the adjoint of the following resample, re-rounded to bf16 as the adjoint kernel
  // stores it)
  auto dy_row = [&](int px) -> uint4 {
    if constexpr (RS) {
      if (dyrs) {
        float v[8];
        gn_resample_adj(DY, p.lddy, dyrs, p.w, px, v);
        return pack8(v);
      }
    }
    return *(const uint4*)(DY + (long)px * p.lddy);
  };
  const bf16_t* RSA = RS && rsrs ? (const bf16_t*)p.resid + (long)L.b * gn_rs_hw(rsrs, HW) * p.ld_resid + L.cb
                                 : nullptr;
  const bf16_t* DSR = DSL ? (const bf16_t*)p.dsilu + off * p.ld_dsilu + L.cb : nullptr;
  // per-channel constants
  float xm[8], xr[8], ga[8], be[8], sc1[8], sf[8];
  load8f(p.gamma + L.cb, ga);
  load8f(p.beta + L.cb, be);
  if (film) {
    load8f(p.film + (long)L.b * p.ld_film + L.cb, sc1);
    load8f(p.film + (long)L.b * p.ld_film + p.c + L.cb, sf);
  }
  const float* st = p.stats + ((long)L.b * p.groups) * 2;
  // z = xhat * zg + zb (gamma and the FiLM scale folded), xhat = x * xr + xo; pass 2's dn * gamma =
  // dz * sg
  float zg[8], zb[8], xo[8], sg[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = (L.cb + i) / L.cpg;
    xm[i] = st[2 * g]; xr[i] = st[2 * g + 1];
    sc1[i] = film ? 1.f + sc1[i] : 1.f;
    sf[i] = film ? sf[i] : 0.f;
    zg[i] = ga[i] * sc1[i];
    zb[i] = be[i] * sc1[i] + sf[i];
    xo[i] = -xm[i] * xr[i];
    sg[i] = sc1[i] * ga[i];
  }
  // the slice's gamma for the group terms: loaded now into registers, stored to LDS after pass 1
  // (a store here would wait for the load before pass 1 issues its own)
  float gam_r[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = threadIdx.x + j * GN_THREADS;
    gam_r[j] = cl < L.cs ? p.gamma[L.c0 + cl] : 0.f;
  }
  GN_STAMP(2);
  bf16_t* DX = (bf16_t*)p.dx + off * p.lddx + L.cb;
  const bool accum = p.accumulate_dx;
  const bf16_t* RES = p.resid && !RSA ? (const bf16_t*)p.resid + off * p.ld_resid + L.cb : nullptr;
  // rows per batch: every load of a batch issued before the first use (a slab row already has up
  // to 8 loads in flight)
  constexpr int U1 = SLAB ? ED_GN_SLAB_U : ED_GN_BWD_U;
  // ONE: the thread's rows are a single batch (every level at B = 128 but 16x16 x 192): pass 1
  // keeps dn and xhat of its rows in registers and issues pass 2's global operand (skip-branch
  // gradient / the dx being accumulated) with its own loads, before the reductions, so pass 2 is
  // three FMAs and a store per element instead of a second load round trip and a recompute of
  // the SiLU gradient.  (Issuing these loads ahead of the per-channel constants measured no gain.)
  constexpr bool CACHE = !SLAB;
  const bool one = CACHE && HW <= U1 * L.np;
  float cdz[U1][8], cxh[U1][8];
  uint4 gr0[U1];
  // pass 1: per-channel sums of dz and dz*xhat -- the four the backward needs follow from them per
  // channel (dn = dz * s with s = 1 + FiLM scale constant over the image, n = xhat * gamma + beta):
  // sum dn = s sum dz, sum dn*xhat = s sum dz*xhat, sum dz*n = gamma sum dz*xhat + beta sum dz.
  // (Four accumulators cost pass 1 three more VALU ops per element and the reduction twice the
  // shuffles / LDS rows; pass 1 is VALU-bound.)
  float acc[2][8];
#pragma unroll
  for (int k = 0; k < 2; ++k)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[k][i] = 0.f;
  auto row1 = [&](const uint4 ux, const uint4 ud, const uint4 us, const int u, const bool keep) {
    float v[8], d[8], sg1[8];
    unpack8(ux, v);
    unpack8(ud, d);
    if constexpr (DSL) unpack8(us, sg1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xh = v[i] * xr[i] + xo[i];
      float dz;
      if constexpr (DSL) {
        dz = d[i] * sg1[i];
      } else {
        const float z = xh * zg[i] + zb[i];
        dz = silu ? d[i] * silu_grad(z) : d[i];
      }
      acc[0][i] += dz; acc[1][i] += dz * xh;
      if (keep) { cdz[u][i] = dz; cxh[u][i] = xh; }
    }
  };
  if (L.active) {
    if (one) {
      uint4 bx[U1], bd[U1], bs[U1];
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        const int px = L.tp + u * L.np;
        bx[u] = bd[u] = bs[u] = gr0[u] = (uint4){0u, 0u, 0u, 0u};
        if (px < HW) {
          bx[u] = *(const uint4*)(X + (long)px * p.ldx);
          bd[u] = dy_row(px);
          if constexpr (DSL) bs[u] = *(const uint4*)(DSR + (long)px * p.ld_dsilu);
          if (RES) gr0[u] = *(const uint4*)(RES + (long)px * p.ld_resid);
          else if (accum) gr0[u] = *(const uint4*)(DX + (long)px * p.lddx);
        }
      }
#pragma unroll
      for (int u = 0; u < U1; ++u) {
        if (L.tp + u * L.np < HW) row1(bx[u], bd[u], bs[u], u, true);
      }
    } else {
      for (int px0 = L.tp; px0 < HW; px0 += U1 * L.np) {
        uint4 bx[U1], bd[U1], bs[U1];
#pragma unroll
        for (int u = 0; u < U1; ++u) {
          const int px = px0 + u * L.np;
          bx[u] = bd[u] = bs[u] = (uint4){0u, 0u, 0u, 0u};
          if (px < HW) {
            bx[u] = *(const uint4*)(X + (long)px * p.ldx);
            if constexpr (DSL) bs[u] = *(const uint4*)(DSR + (long)px * p.ld_dsilu);
            if constexpr (SLAB) {  // dy combined from its producer's slabs and written back
              bd[u] = gn_slab_row(sl, off + px, p.c, L.cb);
              *(uint4*)(const_cast<bf16_t*>(DY) + (long)px * p.lddy) = bd[u];
            } else {
              bd[u] = dy_row(px);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < U1; ++u) {
          const int px = px0 + u * L.np;
          if (px >= HW) break;
          if (L.tiled) { tx[px * L.nvc + L.tv] = bx[u]; td[px * L.nvc + L.tv] = bd[u]; }
          row1(bx[u], bd[u], bs[u], u, false);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cl = threadIdx.x + j * GN_THREADS;
    if (cl < L.cs) gam_sh[cl] = gam_r[j];
  }
  GN_STAMP(3);
  slice_reduce<2>(acc, L, red, chs);
  GN_STAMP(4);
  // per-channel outputs + gamma-weighted sums for the group terms.  (Threads owning a whole group
  // -- channel totals, partials and group terms behind ONE barrier -- measured slower: +0.3 us at
  // cpg 2, +3.5 us at cpg 16, the few group threads' serial loops outweigh the two barriers.)
  float* gch = red;  // [2][cs] (red is free after the reduction)
  for (int cl = threadIdx.x; cl < L.cs; cl += GN_THREADS) {
    const int c = L.c0 + cl;
    const float gam = gam_sh[cl];
    const float sdz = chs[cl], sdzx = chs[L.cs + cl];
    const float s = film ? 1.f + p.film[(long)L.b * p.ld_film + c] : 1.f;
    const float sdn = s * sdz, sdnx = s * sdzx;
    p.dbeta_part[(long)L.b * p.ld_part + c] = sdn;
    p.dgamma_part[(long)L.b * p.ld_part + c] = sdnx;
    if (film) {
      p.dfilm[(long)L.b * p.ld_dfilm + c] = gam * sdzx + p.beta[c] * sdz;  // d scale = sum dz * n
      p.dfilm[(long)L.b * p.ld_dfilm + p.c + c] = sdz;                    // d shift = sum dz
    }
    gch[cl] = gam * sdn;
    gch[L.cs + cl] = gam * sdnx;
  }
  __syncthreads();
  // group sums by one thread per group (a per-thread sum over the group's channels instead, with no
  // barrier, measured slower: a dependent chain of cpg LDS reads per thread, +0.2 .. +1 us)
  float* gsh = red + 2 * L.cs;  // [2][64]
  if (threadIdx.x < L.gs) {
    float s1 = 0.f, s2 = 0.f;
    for (int cl = threadIdx.x * L.cpg; cl < (threadIdx.x + 1) * L.cpg; ++cl) {
      s1 += gch[cl];
      s2 += gch[L.cs + cl];
    }
    gsh[threadIdx.x] = s1 * inv_n;
    gsh[64 + threadIdx.x] = s2 * inv_n;
  }
  __syncthreads();
  if (!L.active) return;
  float m1[8], m2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int g = (L.tv * 8 + i) / L.cpg;
    m1[i] = gsh[g]; m2[i] = gsh[64 + g];
  }
  GN_STAMP(5);
  auto out_row = [&](const int px, const uint4 g, const float (&dz)[8], const float (&xh)[8]) {
    float o[8];
    if (RES && accum) {  // both: dx (in place) + resid
      float rr[8];
      unpack8(*(const uint4*)(DX + (long)px * p.lddx), o);
      unpack8(g, rr);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] += rr[i];
    } else if (RES || accum) {
      unpack8(g, o);  // residual-branch gradient (skip connection) or the dx being accumulated
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float r = xr[i] * (dz[i] * sg[i] - m1[i] - xh[i] * m2[i]);
      o[i] = (accum || RES) ? o[i] + r : r;
    }
    if constexpr (RS) {
      if (RSA) {  // + the adjoint of the skip branch's resample, after dx's own rounding (as the
                  // separate accumulate pass it replaces added it)
        float a[8];
        gn_resample_adj(RSA, p.ld_resid, rsrs, p.w, px, a);
        unpack8(pack8(o), o);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += a[i];
      }
    }
    *(uint4*)(DX + (long)px * p.lddx) = pack8(o);
  };
  if (one) {
#pragma unroll
    for (int u = 0; u < U1; ++u) {
      const int px = L.tp + u * L.np;
      if (px < HW) out_row(px, gr0[u], cdz[u], cxh[u]);
    }
  } else {
    // U rows per thread: the global (resid / accumulate) reads of all U are issued before the
    // first dx store -- one latency per U rows instead of one per row
    constexpr int U = ED_GN_BWD_U;
    for (int px0 = L.tp; px0 < HW; px0 += U * L.np) {
      uint4 gr[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int px = px0 + u * L.np;
        gr[u] = (uint4){0u, 0u, 0u, 0u};
        if (px < HW) {
          if (RES) gr[u] = *(const uint4*)(RES + (long)px * p.ld_resid);
          else if (accum) gr[u] = *(const uint4*)(DX + (long)px * p.lddx);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int px = px0 + u * L.np;
        if (px >= HW) break;
        float v[8], d[8], dz[8], xh[8], sg1[8];
        unpack8(gn_row(L, tx, X, p.ldx, px), v);
        unpack8(RS && dyrs && !L.tiled ? dy_row(px) : gn_row(L, td, DY, p.lddy, px), d);
        if constexpr (DSL) unpack8(*(const uint4*)(DSR + (long)px * p.ld_dsilu), sg1);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[i] = v[i] * xr[i] + xo[i];
          if constexpr (DSL) {
            dz[i] = d[i] * sg1[i];
          } else {
            const float z = xh[i] * zg[i] + zb[i];
            dz[i] = silu ? d[i] * silu_grad(z) : d[i];
          }
        }
        out_row(px, gr[u], dz, xh);
      }
    }
  }
  GN_STAMP(6);
  GN_STAMP_RT(7);
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
__global__ __launch_bounds__(256) void ln_bwd_kernel(const EncdiffLayerNormArgs p, const GnSlabs sl) {
  constexpr int LPR = C / 8;
  constexpr int RPB = 256 / LPR;
  __shared__ float red[2][RPB][C];
  const int lr = threadIdx.x % LPR;
  const int rr = threadIdx.x / LPR;
  float ga[8], dga[8], dbe[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) { ga[i] = p.gamma[lr * 8 + i]; dga[i] = 0.f; dbe[i] = 0.f; }
  // U rows per thread in flight: every load of all U is issued before any store (the stores to
  // dx may alias the loaded tensors, so the compiler would not hoist them itself).  (4 -- one load
  // round trip for the step's c = 64 calls instead of two -- measured slower: 256+ VGPRs)
  constexpr int U = ED_LN_BWD_U;
  const int stride = gridDim.x * RPB;
  for (int row0 = blockIdx.x * RPB + rr; row0 < p.rows; row0 += U * stride) {
    float v[U][8], d[U][8], o8[U][8], mean[U], rstd[U];
    bool rp_on[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * stride;
      rp_on[u] = false;
      if (row >= p.rows) continue;
      unpack8(*(const uint4*)((const bf16_t*)p.x + (long)row * p.ldx + lr * 8), v[u]);
      if (sl.ws) {  // dy combined from its producer's slabs and written back
        const uint4 du = gn_slab_row(sl, row, C, lr * 8);
        *(uint4*)((bf16_t*)p.dy + (long)row * p.lddy + lr * 8) = du;
        unpack8(du, d[u]);
      } else {
        unpack8(*(const uint4*)((const bf16_t*)p.dy + (long)row * p.lddy + lr * 8), d[u]);
      }
      mean[u] = p.stats[2 * row];
      rstd[u] = p.stats[2 * row + 1];
      // residual-branch gradient: dx itself (in place) or a separate tensor (out of place, so a
      // weight gradient still reading that tensor on another stream is not overwritten)
      const bf16_t* rp = p.resid ? (const bf16_t*)p.resid + (long)row * p.ld_resid + lr * 8
                                 : (p.accumulate_dx ? (const bf16_t*)p.dx + (long)row * p.lddx + lr * 8 : nullptr);
      if (rp) { unpack8(*(const uint4*)rp, o8[u]); rp_on[u] = true; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = row0 + u * stride;
      if (row >= p.rows) continue;  // (uniform across the row's LPR lanes)
      float s1 = 0.f, s2 = 0.f, xh[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        xh[i] = (v[u][i] - mean[u]) * rstd[u];
        const float g = d[u][i] * ga[i];
        s1 += g; s2 += g * xh[i];
        dga[i] += d[u][i] * xh[i];
        dbe[i] += d[u][i];
      }
#pragma unroll
      for (int o = LPR / 2; o > 0; o >>= 1) { s1 += __shfl_xor(s1, o, 64); s2 += __shfl_xor(s2, o, 64); }
      s1 *= (1.f / C); s2 *= (1.f / C);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float r = rstd[u] * (d[u][i] * ga[i] - s1 - xh[i] * s2);
        o8[u][i] = rp_on[u] ? o8[u][i] + r : r;
      }
      *(uint4*)((bf16_t*)p.dx + (long)row * p.lddx + lr * 8) = pack8(o8[u]);
    }
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

// channel-slice width: the narrowest multiple of lcm(8, channels-per-group) dividing C whose
// slice holds >= gn_min_slice() elements (so small images still fill a workgroup), else all of C.
int gn_min_slice() {
  static const int v = [] {
    const char* e = getenv("ENCDIFF_GN_MIN_SLICE");  // tuning knob (elements per workgroup)
    return e ? atoi(e) : 8192;  // measured best of 1K..64K on the step's shapes (tools/kbench.py)
  }();
  return v;
}

// small batches (sampling) keep more workgroups: a quarter of the slice size below 64 images
int gn_slice(int C, int HW, int cpg, int batch) {
  int unit = 8;
  while (unit % cpg) unit += 8;
  // smaller images: smaller slices (more workgroups); measured per UNet level with
  // tools/gn_bench.py: 8K elements at 16x16, 4K at 8x8, 2K at 4x4, 1K at 2x2
  const int shrink = HW >= 256 ? 1 : (HW >= 64 ? 2 : (HW >= 16 ? 4 : 8));
  const long min_el = (batch >= 64 ? gn_min_slice() : gn_min_slice() / 4) / shrink;
  // (a smaller slice that fits the backward's LDS tile at 16x16 x 192 channels -- 24 instead of
  // 48 channels, non-power-of-two lane reduction -- measured slower: 23.4 -> 26.3 us)
  for (int w = unit; w < C; w += unit)
    if (C % w == 0 && (long)w * HW >= min_el) return w;
  return C;
}

// slabs of a GEMM whose deferred finalize output is the tensor t (ld) a GroupNorm reads
int gn_slabs_of(const EncdiffGemmArgs& g, const void* t, long ld, const EncdiffGroupNormArgs* a, GnSlabs& sl) {
  const bool tp = g.a_mode == ENCDIFF_OPA_IM2COL && g.conv.resample == ENCDIFF_RESAMPLE_K4S2_TP;
  if (g.dtype != ENCDIFF_DT_BF16 || g.c_mode != ENCDIFF_OUT_BF16 || g.split_k < 2 || !g.workspace ||
      g.split_counters || g.bias_grad || tp || g.c != t || g.ldc != ld || g.N != a->c ||
      (long)g.M != (long)a->batch * a->hw || ((uintptr_t)g.workspace & 15) || (g.bias && ((uintptr_t)g.bias & 15)) ||
      (g.resid && (g.ld_resid % 8 || ((uintptr_t)g.resid & 15))))
    return ENCDIFF_ERR_ARG;
  sl = GnSlabs{g.workspace, (long)g.M * g.N, g.split_k, g.alpha, g.bias, (const bf16_t*)g.resid, g.ld_resid};
  return ENCDIFF_OK;
}

int gn_check(const EncdiffGroupNormArgs* a) {
  if (a->c % 8 || a->groups <= 0 || a->c % a->groups) return ENCDIFF_ERR_SHAPE;
  const int cs = gn_slice(a->c, a->hw, a->c / a->groups, a->batch);
  if (cs > 512 || cs / (a->c / a->groups) > 64) return ENCDIFF_ERR_UNSUPPORTED;
  return cs;
}

}  // namespace

extern "C" int encdiff_groupnorm_fwd(const EncdiffGroupNormArgs* a, void* stream) {
  if (a && a->dtype == ENCDIFF_DT_F32) return a->x_from ? ENCDIFF_ERR_UNSUPPORTED : ed_groupnorm_fwd_f32(a, (hipStream_t)stream);
  if (!a || a->dtype != ENCDIFF_DT_BF16 || !a->x || !a->y || !a->stats || !a->gamma || !a->beta) return ENCDIFF_ERR_ARG;
  if (a->silu && a->dsilu && (((uintptr_t)a->dsilu & 15) || a->ld_dsilu % 8)) return ENCDIFF_ERR_ARG;
  const int cs = gn_check(a);
  if (cs < 0) return cs;
  GnSlabs sl{};
  if (a->x_from) {  // x = the deferred split-K finalize of its producer (self-reducing kernel only)
    if (a->in_stats) return ENCDIFF_ERR_ARG;
    const int rc = gn_slabs_of(*a->x_from, a->x, a->ldx, a, sl);
    if (rc != ENCDIFF_OK) return rc;
  }
  // producer statistics feed the two statistics kernels where their layout fits; other
  // shapes (e.g. a 384-channel concat at 32x32) take the self-reducing kernel below
  const bool st_ok = a->in_stats && a->hw % 64 == 0 && a->ld_in_stats >= a->c;
  if (st_ok && a->hw >= 1024 && a->c <= 512 && a->groups <= 64 && GN_THREADS % (a->c >> 3) == 0) {
    // large images: group-statistics kernel + streaming apply
    hipLaunchKernelGGL(gn_group_stats_kernel, dim3(a->batch), dim3(GN_THREADS), 0, (hipStream_t)stream, *a);
    const int rpb = 256;
    hipLaunchKernelGGL(gn_apply_kernel, dim3((a->hw + rpb - 1) / rpb, a->batch), dim3(GN_THREADS), 0,
                       (hipStream_t)stream, *a, rpb);
    ED_CHECK_LAUNCH();
    return ENCDIFF_OK;
  }
  if (st_ok && (a->hw / 64) * cs <= 2048) {  // statistics from the producer GEMM's segment sums
    hipLaunchKernelGGL(gn_fwd_stats_kernel, dim3(a->batch * (a->c / cs)), dim3(GN_THREADS), 0, (hipStream_t)stream,
                       *a, cs);
    ED_CHECK_LAUNCH();
    return ENCDIFF_OK;
  }
  const long need = (long)(cs / 8) * a->hw;  // 16-byte vectors of one slice
  const int cap = need <= GN_TILE_FWD ? (int)need : 0;
  static const hipError_t attr = hipFuncSetAttribute((const void*)gn_fwd_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
  (void)attr;
  hipLaunchKernelGGL(gn_fwd_kernel, dim3(a->batch * (a->c / cs)), dim3(GN_THREADS), (size_t)cap * 16,
                     (hipStream_t)stream, *a, cs, cap, sl);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

#if ED_GN_STAMP
extern "C" int encdiff_debug_gn_stamps(void* dst, int nblocks) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(gn_stamps), (size_t)nblocks * 8 * sizeof(unsigned long long)) == hipSuccess
             ? 0 : -1;
}
#endif

extern "C" int encdiff_groupnorm_bwd(const EncdiffGroupNormArgs* a, void* stream) {
  if (a && a->dtype == ENCDIFF_DT_F32 && a->fold_plan) return ENCDIFF_ERR_UNSUPPORTED;
  if (a && a->dtype == ENCDIFF_DT_F32)
    return (a->dy_resample || a->resid_resample) ? ENCDIFF_ERR_UNSUPPORTED : ed_groupnorm_bwd_f32(a, (hipStream_t)stream);
  if (a && a->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_UNSUPPORTED;
  if (!a || !a->x || !a->dy || !a->dx || !a->stats || !a->dgamma_part || !a->dbeta_part) return ENCDIFF_ERR_ARG;
  if (a->film && !a->dfilm) return ENCDIFF_ERR_ARG;
  const int cs = gn_check(a);
  if (cs < 0) return cs;
  GnSlabs sl{};
  if (a->x_from) {  // dy = the deferred split-K finalize of its producer
    const int rc = gn_slabs_of(*a->x_from, a->dy, a->lddy, a, sl);
    if (rc != ENCDIFF_OK) return rc;
  }
  if ((a->fold_plan != nullptr) != (a->fold_blocks > 0) || a->fold_blocks < 0) return ENCDIFF_ERR_ARG;
  const int fold = a->fold_plan ? a->fold_blocks : 0;
  const bool rs = a->dy_resample || a->resid_resample;
  const bool dsl = a->silu && a->dsilu != nullptr;
  // dynamic LDS: pixel tiles only where pass 2 reads them (not register-cached single-batch slices,
  // gn_bwd_kernel's `one`), reduction rows (slice_partials: 4 wave rows for power-of-two vector
  // counts, one per pixel lane otherwise; >= the group-term scratch [2][cs] + [2][64] and the fold's
  // [8][32] float4)
  const int nvc = cs / 8, np = GN_THREADS / nvc;
  const bool one = !sl.ws && a->hw <= ED_GN_BWD_U * np;
  const int ntile = (!one && nvc * a->hw <= GN_TILE) ? nvc * a->hw : 0;
  const bool pow2 = (nvc & (nvc - 1)) == 0;
  const int rows = pow2 ? (nvc >= 64 ? GN_THREADS / nvc : GN_THREADS / 64) : np;
  int nred = std::max(rows * 2 * cs, 2 * cs + 128);
  if (a->fold_plan) nred = std::max(nred, 8 * 32 * 4);
  nred = (nred + 3) & ~3;
#if GN_BWD_LDS_FULL  // A/B: the former static sizing (tiles for every tiled slice, 8192 reduction floats)
  const int ntile_ = nvc * a->hw <= GN_TILE ? GN_TILE : 0;
  nred = 4 * 2048;
#else
  const int ntile_ = ntile;
#endif
  const size_t lds = (size_t)2 * ntile_ * 16 + (size_t)(nred + 3 * cs) * 4;
  if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
  static const bool attr_ok = [] {
    const void* ks[] = {(const void*)gn_bwd_kernel<false>, (const void*)gn_bwd_kernel<true>,
                        (const void*)gn_bwd_kernel<false, true>, (const void*)gn_bwd_kernel<false, false, true>,
                        (const void*)gn_bwd_kernel<true, false, true>, (const void*)gn_bwd_kernel<false, true, true>};
    bool ok = true;
    for (const void* k : ks) ok = ok && hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
    return ok;
  }();
  if (!attr_ok) return ENCDIFF_ERR_LAUNCH;
  if (dsl && (((uintptr_t)a->dsilu & 15) || a->ld_dsilu % 8)) return ENCDIFF_ERR_ARG;
  if (rs) {  // operands at a following resample's resolution (read through its adjoint)
    auto ok_mode = [](int m) { return m == 0 || m == ENCDIFF_RESAMPLE_DOWN2 || m == ENCDIFF_RESAMPLE_UP2; };
    if (!ok_mode(a->dy_resample) || !ok_mode(a->resid_resample) || sl.ws || a->w <= 0 || a->hw % a->w ||
        (a->resid_resample && !a->resid))
      return ENCDIFF_ERR_ARG;
    const int h = a->hw / a->w;
    if ((a->dy_resample == ENCDIFF_RESAMPLE_DOWN2 || a->resid_resample == ENCDIFF_RESAMPLE_DOWN2) && ((h | a->w) & 1))
      return ENCDIFF_ERR_SHAPE;
    if (dsl)
      hipLaunchKernelGGL((gn_bwd_kernel<false, true, true>), dim3(a->batch * (a->c / cs) + fold), dim3(GN_THREADS), lds,
                         (hipStream_t)stream, *a, cs, sl, ntile_, nred);
    else
      hipLaunchKernelGGL((gn_bwd_kernel<false, true>), dim3(a->batch * (a->c / cs) + fold), dim3(GN_THREADS), lds,
                         (hipStream_t)stream, *a, cs, sl, ntile_, nred);
  } else if (sl.ws) {
    if (dsl)
      hipLaunchKernelGGL((gn_bwd_kernel<true, false, true>), dim3(a->batch * (a->c / cs) + fold), dim3(GN_THREADS), lds,
                         (hipStream_t)stream, *a, cs, sl, ntile_, nred);
    else
      hipLaunchKernelGGL(gn_bwd_kernel<true>, dim3(a->batch * (a->c / cs) + fold), dim3(GN_THREADS), lds, (hipStream_t)stream,
                         *a, cs, sl, ntile_, nred);
  } else {
    if (dsl)
      hipLaunchKernelGGL((gn_bwd_kernel<false, false, true>), dim3(a->batch * (a->c / cs) + fold), dim3(GN_THREADS), lds,
                         (hipStream_t)stream, *a, cs, sl, ntile_, nred);
    else
      hipLaunchKernelGGL(gn_bwd_kernel<false>, dim3(a->batch * (a->c / cs) + fold), dim3(GN_THREADS), lds,
                         (hipStream_t)stream, *a, cs, sl, ntile_, nred);
  }
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

template <int C>
static int ln_launch(const EncdiffLayerNormArgs& a, bool bwd, hipStream_t s) {
  constexpr int RPB = 256 / (C / 8);
  if (bwd) {
    GnSlabs sl{};
    if (a.dy_from) {  // dy = the deferred split-K finalize of its producer (same checks as GroupNorm's)
      const EncdiffGemmArgs& g = *a.dy_from;
      if (g.dtype != ENCDIFF_DT_BF16 || g.c_mode != ENCDIFF_OUT_BF16 || g.split_k < 2 || !g.workspace ||
          g.split_counters || g.bias_grad || g.a_mode == ENCDIFF_OPA_IM2COL || g.c != a.dy || g.ldc != a.lddy ||
          g.N != C || g.M != a.rows || ((uintptr_t)g.workspace & 15) || (g.bias && ((uintptr_t)g.bias & 15)) ||
          (g.resid && (g.ld_resid % 8 || ((uintptr_t)g.resid & 15))))
        return ENCDIFF_ERR_ARG;
      sl = GnSlabs{g.workspace, (long)g.M * g.N, g.split_k, g.alpha, g.bias, (const bf16_t*)g.resid, g.ld_resid};
    }
    hipLaunchKernelGGL(ln_bwd_kernel<C>, dim3(a.parts), dim3(256), 0, s, a, sl);
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

extern "C" int encdiff_layernorm_fwd(const EncdiffLayerNormArgs* a, void* stream) {
  if (a && a->dtype == ENCDIFF_DT_F32) return ed_layernorm_fwd_f32(a, (hipStream_t)stream);
  if (a && a->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_ARG;
  return ln_dispatch(a, false, stream);
}
extern "C" int encdiff_layernorm_bwd(const EncdiffLayerNormArgs* a, void* stream) {
  if (a && a->dtype == ENCDIFF_DT_F32) return ed_layernorm_bwd_f32(a, (hipStream_t)stream);
  if (a && a->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_UNSUPPORTED;
  return ln_dispatch(a, true, stream);
}
