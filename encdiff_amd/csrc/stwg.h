// stwg.h -- the grouped weight-gradient plan of a fused transformer block (encdiff_st_wgrad_plan,
// st_bwd.hip) and its chunk fold, shared with the GroupNorm backward (norm.hip), which can carry the
// fold's workgroups in its own grid.
#pragma once
#include "common.h"

namespace {

struct StWg {
  const bf16_t* dy; const bf16_t* x; float* dw; float* db; float* slab;
  long ld_dy, ld_x, ld_dw;
  int M, N, K, kc, kb, mb, nb, item0, fold0, kind, bm, bn;
};
struct StWgHead {
  int magic, nprob, nitems, nfold;
  long probs_off, bytes;
};
constexpr int STWG_MAGIC = 0x53545747;  // "STWG"
constexpr int STWG_MAXP = 16;
#ifndef STWG_FOLD_UNROLL
#define STWG_FOLD_UNROLL 4
#endif

// dW += sum_z slab[z] (and db), fold block `bid` of the plan: a workgroup (256 threads) owns 32 float4
// of one problem's dW (or 32 bias entries); its 8 thread groups sum chunks z = g, g + 8, ...
// (independent loads in flight), and the 8 group sums are added in group order through LDS -- a
// fixed order, reproducible.  Every thread of the workgroup must call it (one barrier).
ED_DEV void stwg_fold_block(const StWg* __restrict__ probs, int nprob, int bid, float4 (*red)[32]) {
  int pi = 0;
  for (int q = 1; q < nprob; ++q)
    if (bid >= probs[q].fold0) pi = q;
  const StWg p = probs[pi];
  if (p.kb == 1) return;
  const int g = threadIdx.x >> 5, l = threadIdx.x & 31;
  const long n4 = (long)p.M * p.N / 4;
  const long nw = (n4 + 31) / 32;  // workgroups of the weight part
  const long blk = bid - p.fold0;
  const long MN = (long)p.M * p.N;
  if (blk < nw) {
    const long e = blk * 32 + l;
    float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < n4) {
      const float* s = p.slab + 4 * e;
#pragma unroll STWG_FOLD_UNROLL
      for (int z = g; z < p.kb; z += 8) {
        const float4 v = *(const float4*)(s + (long)z * MN);
        a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
      }
    }
    red[g][l] = a;
    __syncthreads();
    if (g == 0 && e < n4) {
      float4 t = red[0][l];
#pragma unroll
      for (int k = 1; k < 8; ++k) {
        const float4 v = red[k][l];
        t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w;
      }
      const long m = 4 * e / p.N, n = 4 * e % p.N;
      float* o = p.dw + m * p.ld_dw + n;
      o[0] += t.x; o[1] += t.y; o[2] += t.z; o[3] += t.w;
    }
  } else if (p.db) {  // bias: 32 entries per workgroup, the same group split
    const long m = (blk - nw) * 32 + l;
    float a = 0.f;
    if (m < p.M)
      for (int z = g; z < p.kb; z += 8) a += p.slab[(long)p.kb * MN + (long)z * p.M + m];
    red[g][l].x = a;
    __syncthreads();
    if (g == 0 && m < p.M) {
      float t = red[0][l].x;
#pragma unroll
      for (int k = 1; k < 8; ++k) t += red[k][l].x;
      p.db[m] += t;
    }
  }
}

// the fold block of a plan handed over as its device blob (EncdiffGroupNormArgs.fold_plan)
ED_DEV void stwg_fold_from_blob(const void* blob, int bid, float4 (*red)[32]) {
  const StWgHead* h = (const StWgHead*)blob;
  stwg_fold_block((const StWg*)((const char*)blob + h->probs_off), h->nprob, bid, red);
}

}  // namespace
