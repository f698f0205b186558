// attn.hip -- multi-head attention of the SpatialTransformer (attention.py:170-193).
//
// q/k/v/o are [rows][ld] bf16 with head h at columns [h*dh, (h+1)*dh) ('b n (h d)'),
// read in place (no head split/merge copies).  One workgroup holds `hpb` heads of one
// image: their K and V tiles are staged in LDS (fp32), each thread owns one query row
// and runs an exact online softmax over the keys (fp32), writing O and the row
// log-sum-exp.  The backward recomputes P from the saved LSE: phase 1 (thread per
// query) produces dQ and the row terms D = rowsum(dO*O); phase 2 (thread per key)
// produces dK and dV -- no atomics, no score matrix in HBM.
// Sizes on the path: self S in {256, 64, 16, 4} with dh {8, 16, 32, 32}, cross Sk = 20.
#include "common.h"

int encdiff_attention_mfma(const EncdiffAttnArgs* a, bool bwd, void* stream);

namespace {

ED_DEV void load_row(const bf16_t* __restrict__ src, int dh, float* dst) {
  // dh in {8, 16, 32}: 16-byte vectors
  for (int d = 0; d < dh; d += 8) {
    float v[8];
    unpack8(*(const uint4*)(src + d), v);
#pragma unroll
    for (int i = 0; i < 8; ++i) dst[d + i] = v[i];
  }
}

template <int DH>
__global__ __launch_bounds__(256) void attn_fwd_kernel(const EncdiffAttnArgs p, int hpb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = p.heads, SQ = p.sq, SK = p.sk;
  const int bh0 = blockIdx.x * hpb;          // first (b*H + h) of this block
  float* Ks = sm;                             // [hpb][SK][DH]
  float* Vs = sm + hpb * SK * DH;
  // stage K, V
  for (int idx = threadIdx.x; idx < hpb * SK; idx += blockDim.x) {
    const int hl = idx / SK, j = idx - hl * SK;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    load_row((const bf16_t*)p.k + ((long)b * SK + j) * p.ldk + h * DH, DH, Ks + idx * DH);
    load_row((const bf16_t*)p.v + ((long)b * SK + j) * p.ldv + h * DH, DH, Vs + idx * DH);
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t >= hpb * SQ) return;
  const int hl = t / SQ, qi = t - hl * SQ;
  const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
  float q[DH], o[DH];
  load_row((const bf16_t*)p.q + ((long)b * SQ + qi) * p.ldq + h * DH, DH, q);
#pragma unroll
  for (int d = 0; d < DH; ++d) { q[d] *= p.scale; o[d] = 0.f; }
  float m = -INFINITY, l = 0.f;
  const float* kb = Ks + hl * SK * DH;
  const float* vb = Vs + hl * SK * DH;
  for (int j = 0; j < SK; ++j) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) s += q[d] * kb[j * DH + d];
    if (s > m) {
      const float a = __expf(m - s);
      l *= a;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] *= a;
      m = s;
    }
    const float e = __expf(s - m);
    l += e;
#pragma unroll
    for (int d = 0; d < DH; ++d) o[d] += e * vb[j * DH + d];
  }
  const float inv = 1.f / l;
  bf16_t* op = (bf16_t*)p.o + ((long)b * SQ + qi) * p.ldo + h * DH;
#pragma unroll
  for (int d = 0; d < DH; d += 8) {
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = o[d + i] * inv;
    *(uint4*)(op + d) = pack8(v);
  }
  if (p.lse) p.lse[(long)bh * SQ + qi] = m + __logf(l);
}

template <int DH>
__global__ __launch_bounds__(256) void attn_bwd_kernel(const EncdiffAttnArgs p, int hpb) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int H = p.heads, SQ = p.sq, SK = p.sk;
  const int bh0 = blockIdx.x * hpb;
  float* Ks = sm;                          // [hpb][SK][DH]
  float* Vs = Ks + hpb * SK * DH;
  float* Qs = Vs + hpb * SK * DH;          // [hpb][SQ][DH] (scaled q)
  float* Gs = Qs + hpb * SQ * DH;          // [hpb][SQ][DH] dO
  float* Ls = Gs + hpb * SQ * DH;          // [hpb][SQ] lse
  float* Ds = Ls + hpb * SQ;               // [hpb][SQ] rowsum(dO*O)
  for (int idx = threadIdx.x; idx < hpb * SK; idx += blockDim.x) {
    const int hl = idx / SK, j = idx - hl * SK;
    const int bh = bh0 + hl, b = bh / H, h = bh - b * H;
    load_row((const bf16_t*)p.k + ((long)b * SK + j) * p.ldk + h * DH, DH, Ks + idx * DH);
    load_row((const bf16_t*)p.v + ((long)b * SK + j) * p.ldv + h * DH, DH, Vs + idx * DH);
  }
  // phase 1: thread per query -> dQ, D
  const int t = threadIdx.x;
  float q[DH], g[DH];
  int hl = 0, qi = 0, b = 0, h = 0;
  const bool qact = t < hpb * SQ;
  if (qact) {
    hl = t / SQ; qi = t - hl * SQ;
    const int bh = bh0 + hl; b = bh / H; h = bh - b * H;
    float o[DH];
    load_row((const bf16_t*)p.q + ((long)b * SQ + qi) * p.ldq + h * DH, DH, q);
    load_row((const bf16_t*)p.d_o + ((long)b * SQ + qi) * p.lddo + h * DH, DH, g);
    load_row((const bf16_t*)p.o + ((long)b * SQ + qi) * p.ldo + h * DH, DH, o);
    float D = 0.f;
#pragma unroll
    for (int d = 0; d < DH; ++d) { D += g[d] * o[d]; q[d] *= p.scale; }
    const float lse = p.lse[(long)bh * SQ + qi];
    Ls[t] = lse; Ds[t] = D;
#pragma unroll
    for (int d = 0; d < DH; ++d) { Qs[t * DH + d] = q[d]; Gs[t * DH + d] = g[d]; }
  }
  __syncthreads();
  if (qact) {
    const float* kb = Ks + hl * SK * DH;
    const float* vb = Vs + hl * SK * DH;
    const float lse = Ls[t], D = Ds[t];
    float dq[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) dq[d] = 0.f;
    for (int j = 0; j < SK; ++j) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) { s += q[d] * kb[j * DH + d]; dp += g[d] * vb[j * DH + d]; }
      const float pr = __expf(s - lse);
      const float ds = pr * (dp - D);
#pragma unroll
      for (int d = 0; d < DH; ++d) dq[d] += ds * kb[j * DH + d];
    }
    bf16_t* dqp = (bf16_t*)p.dq + ((long)b * SQ + qi) * p.lddq + h * DH;
#pragma unroll
    for (int d = 0; d < DH; d += 8) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = dq[d + i] * p.scale;
      *(uint4*)(dqp + d) = pack8(v);
    }
  }
  // phase 2: thread per key -> dK, dV
  for (int kidx = t; kidx < hpb * SK; kidx += blockDim.x) {
    const int khl = kidx / SK, j = kidx - khl * SK;
    const int bh = bh0 + khl, kb_ = bh / H, kh = bh - kb_ * H;
    float k[DH], v[DH], dk[DH], dv[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      k[d] = Ks[kidx * DH + d]; v[d] = Vs[kidx * DH + d]; dk[d] = 0.f; dv[d] = 0.f;
    }
    const float* qb = Qs + khl * SQ * DH;
    const float* gb = Gs + khl * SQ * DH;
    for (int i = 0; i < SQ; ++i) {
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) { s += qb[i * DH + d] * k[d]; dp += gb[i * DH + d] * v[d]; }
      const float pr = __expf(s - Ls[khl * SQ + i]);
      const float ds = pr * (dp - Ds[khl * SQ + i]);
#pragma unroll
      for (int d = 0; d < DH; ++d) { dv[d] += pr * gb[i * DH + d]; dk[d] += ds * qb[i * DH + d]; }
    }
    // q was pre-scaled, so dk already carries the softmax scale
    bf16_t* dkp = (bf16_t*)p.dk + ((long)kb_ * SK + j) * p.lddk + kh * DH;
    bf16_t* dvp = (bf16_t*)p.dv + ((long)kb_ * SK + j) * p.lddv + kh * DH;
#pragma unroll
    for (int d = 0; d < DH; d += 8) {
      *(uint4*)(dkp + d) = pack8(dk + d);
      *(uint4*)(dvp + d) = pack8(dv + d);
    }
  }
}

int heads_per_block(const EncdiffAttnArgs& a) {
  int hpb = 1;
  while (hpb < a.heads && hpb * 2 * a.sq <= 256 && hpb * 2 * a.sk <= 256 && a.heads % (hpb * 2) == 0) hpb *= 2;
  return hpb;
}

template <int DH>
int attn_launch(const EncdiffAttnArgs& a, bool bwd, hipStream_t s) {
  const int hpb = heads_per_block(a);
  const int nblk = a.batch * a.heads / hpb;
  int threads = hpb * (a.sq > a.sk ? a.sq : a.sk);
  threads = ((threads + 63) / 64) * 64;
  if (threads > 256) {
    if (hpb * a.sq > 256) return ENCDIFF_ERR_SHAPE;
    threads = 256;
  }
  if (!bwd) {
    const size_t lds = 2 * hpb * a.sk * DH * sizeof(float);
    hipLaunchKernelGGL(attn_fwd_kernel<DH>, dim3(nblk), dim3(threads), lds, s, a, hpb);
  } else {
    const size_t lds = (2 * hpb * a.sk * DH + 2 * hpb * a.sq * DH + 2 * hpb * a.sq) * sizeof(float);
    if (lds > 160 * 1024) return ENCDIFF_ERR_SHAPE;
    static const hipError_t attr = hipFuncSetAttribute((const void*)attn_bwd_kernel<DH>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)attr;
    hipLaunchKernelGGL(attn_bwd_kernel<DH>, dim3(nblk), dim3(threads), lds, s, a, hpb);
  }
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

int attn_dispatch(const EncdiffAttnArgs* a, bool bwd, void* stream) {
  if (!a || !a->q || !a->k || !a->v || !a->o) return ENCDIFF_ERR_ARG;
  if (bwd && (!a->d_o || !a->dq || !a->dk || !a->dv || !a->lse)) return ENCDIFF_ERR_ARG;
  // MFMA path (attn_mfma.hip) for every shape whose tiles fit LDS; the VALU kernels
  // below remain for head groups too large for one workgroup's LDS.
  const int rc = encdiff_attention_mfma(a, bwd, stream);
  if (rc != ENCDIFF_ERR_SHAPE) return rc;
  if (a->sq > 256) return ENCDIFF_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  switch (a->dh) {
    case 8: return attn_launch<8>(*a, bwd, s);
    case 16: return attn_launch<16>(*a, bwd, s);
    case 32: return attn_launch<32>(*a, bwd, s);
    default: return ENCDIFF_ERR_UNSUPPORTED;
  }
}

}  // namespace

extern "C" int encdiff_attention_fwd(const EncdiffAttnArgs* a, void* stream) { return attn_dispatch(a, false, stream); }
extern "C" int encdiff_attention_bwd(const EncdiffAttnArgs* a, void* stream) { return attn_dispatch(a, true, stream); }
