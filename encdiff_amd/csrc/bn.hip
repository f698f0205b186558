// bn.hip -- training-mode BatchNorm2d (+ReLU) over NHWC activations for the concept
// encoder Encoder4 (openaimodel_enc.py:1002-1012: Conv2d(k4,s2,p1) + BatchNorm2d (+ReLU)
// trunk, EncResBlock(bn=True) at :969-989), and the image repack feeding its first conv.
//
// Statistics are over all N*H*W pixels of a channel (BatchNorm2d.train(), biased variance
// for the normalisation, unbiased for running_var, momentum 0.1).  Each reduction is one
// launch: workgroups reduce a contiguous pixel range into per-workgroup partials, and the
// LAST workgroup to finish (device-scope counter) folds the partials in a fixed order, in
// fp64 -- deterministic, no atomics on data -- and resets the counter for the next launch
// (graph-replay safe).  The elementwise apply is a second launch.
// The pre-BN input x is fp32 (x_f32: the producing conv's fp32 output, so the ReLU masks are
// taken on values as the fp32 reference computes them) or bf16; outputs are bf16.
#include "common.h"

namespace {

constexpr int BN_T = 256;
// workgroups of a reduction (pixel ranges of >= 256 rows, at most 128); ENCDIFF_BN_MAXBLK tunes the cap
// (more workgroups: more loads in flight, longer serial fold in the last one)
int bn_maxblk() {
  static const int v = [] {
    const char* e = getenv("ENCDIFF_BN_MAXBLK");
    const int n = e ? atoi(e) : 128;  // tools/bn_bench.py sweep 64..1024: 128 best at 131K rows
    return n < 1 ? 1 : n;
  }();
  return v;
}

int bn_blocks(int rows) {
  const int b = (rows + 255) / 256;
  return b < bn_maxblk() ? b : bn_maxblk();
}

// 8 consecutive channels of row r of x as fp32: bf16 (one 16-byte load) or fp32 (two)
template <bool F32>
ED_DEV void ld_x8(const void* x, long off, float* v) {
  if constexpr (F32) {
    const float4 a = *(const float4*)((const float*)x + off), b = *(const float4*)((const float*)x + off + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  } else {
    unpack8(*(const uint4*)((const bf16_t*)x + off), v);
  }
}

struct BnLayout {  // thread -> (8-channel vector, pixel lane)
  int nv, lanes, v, pl;
  ED_DEV BnLayout(int c) {
    nv = c >> 3;
    lanes = BN_T / nv;
    v = threadIdx.x % nv;
    pl = threadIdx.x / nv;
  }
};

// 8 per-channel fp32 constants as two 16-byte loads (p is 32-byte aligned: channel offsets
// are multiples of 8 and the per-channel arrays are allocator-aligned); scalar loads made the
// apply kernels issue 33-49 load instructions per 16-byte activation vector
ED_DEV void ld8f(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
  v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

// per-workgroup partial [blk][NQ][c] from q[NQ][8] of every thread: LDS rows summed in order
template <int NQ>
ED_DEV void bn_block_partial(const float (&q)[NQ][8], const BnLayout& L, int c, float* part_out) {
  __shared__ float red[BN_T * 8 * NQ];
  if (L.pl < L.lanes) {
#pragma unroll
    for (int k = 0; k < NQ; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[(k * L.lanes + L.pl) * c + L.v * 8 + i] = q[k][i];
  }
  __syncthreads();
  // write-through (sc1) stores: the partials reach memory without an agent release (which would
  // write back every dirty line of the XCD's L2 in every workgroup) -- bn_last_block
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)part_out, 0, 0x7FFFFFF0, 0x00020000);
  for (int e = threadIdx.x; e < NQ * c; e += BN_T) {
    const int k = e / c, ch = e - k * c;
    float a = 0.f;
    for (int r = 0; r < L.lanes; ++r) a += red[(k * L.lanes + r) * c + ch];
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, a), rs, (int)(((long)k * c + ch) * 4), 0, 16);
  }
}

// fold the per-workgroup partials [nblk][2][c] in a fixed order (fp64): the 2c values of a
// block are c/2 float4 groups; thread t owns group t % (c/2) and sums blocks t / (c/2),
// + J, ... (J = 256 / (c/2) block lanes, 8 loads in flight), then the J lane sums of each
// value are added in lane order through LDS.  Result out[2][c].
ED_DEV void bn_fold(const float* part, int nblk, int c, double* out) {
  __shared__ double fold[4 * BN_T];  // [J][2c]: J * 2c == 4 * 256
  const int V4 = c >> 1, J = BN_T / V4;
  const int g = threadIdx.x % V4, j = threadIdx.x / V4;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll 8
  for (int b = j; b < nblk; b += J) {
    const float4 v = *(const float4*)(part + (long)b * 2 * c + 4 * g);
    a0 += v.x; a1 += v.y; a2 += v.z; a3 += v.w;
  }
  double* f = fold + j * 2 * c + 4 * g;
  f[0] = a0; f[1] = a1; f[2] = a2; f[3] = a3;
  __syncthreads();
  for (int e = threadIdx.x; e < 2 * c; e += BN_T) {
    double t = 0.0;
    for (int k = 0; k < J; ++k) t += fold[k * 2 * c + e];
    out[e] = t;
  }
  __syncthreads();
}

// true in exactly one workgroup: the last to arrive, after every workgroup's partials are
// visible to it (the guide's write-through hand-off: every wave's sc1 partial stores drained,
// a barrier, one lane's agent-scope ticket; the last arriver acquires before reading them)
ED_DEV bool bn_last_block(unsigned int* counter) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == gridDim.x - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return last != 0;
}

template <bool F32>
__global__ __launch_bounds__(BN_T) void bn_stats_kernel(const EncdiffBatchNormArgs p) {
  const BnLayout L(p.c);
  const int per = (p.rows + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(p.rows, r0 + per);
  float q[2][8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[0][i] = q[1][i] = 0.f;
  if (L.pl < L.lanes) {
    // 8 rows (16-byte loads) in flight per thread: one workgroup per CU needs them to cover
    // HBM latency (4 in flight measured ~3 TB/s at 131K rows, tools/bn_bench.py)
#pragma unroll 8
    for (int r = r0 + L.pl; r < r1; r += L.lanes) {
      float x[8];
      ld_x8<F32>(p.x, (long)r * p.ldx + L.v * 8, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) { q[0][i] += x[i]; q[1][i] += x[i] * x[i]; }
    }
  }
  float* part = p.partials + (long)blockIdx.x * 2 * p.c;
  bn_block_partial<2>(q, L, p.c, part);
  if (!bn_last_block(p.counter)) return;
  __shared__ double tot[2 * BN_T];
  bn_fold(p.partials, gridDim.x, p.c, tot);
  const double n = (double)p.rows;
  for (int ch = threadIdx.x; ch < p.c; ch += BN_T) {
    const double s = tot[ch], ss = tot[p.c + ch];
    const double mean = s / n;
    double var = ss / n - mean * mean;
    var = var > 0.0 ? var : 0.0;
    p.mean[ch] = (float)mean;
    p.rstd[ch] = (float)(1.0 / sqrt(var + (double)p.eps));
    if (p.running_mean) {
      const float m = p.momentum;
      p.running_mean[ch] = (1.f - m) * p.running_mean[ch] + m * (float)mean;
      p.running_var[ch] = (1.f - m) * p.running_var[ch] + m * (float)(var * n / (n > 1.0 ? n - 1.0 : 1.0));
    }
  }
  if (threadIdx.x == 0) *p.counter = 0u;
}

template <bool F32>
__global__ __launch_bounds__(BN_T) void bn_apply_kernel(const EncdiffBatchNormArgs p) {
  const int nv = p.c >> 3;
  const int total = p.rows * nv;  // < 2^31 (bn_check): 32-bit index math
  for (int e = blockIdx.x * BN_T + threadIdx.x; e < total; e += gridDim.x * BN_T) {
    const int r = e / nv;
    const int cb = (e - r * nv) * 8;
    float x[8], m[8], rs[8], g[8], b[8];
    ld_x8<F32>(p.x, (long)r * p.ldx + cb, x);
    ld8f(p.mean + cb, m);
    ld8f(p.rstd + cb, rs);
    ld8f(p.gamma + cb, g);
    ld8f(p.beta + cb, b);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float z = (x[i] - m[i]) * rs[i] * g[i] + b[i];
      x[i] = p.relu ? fmaxf(z, 0.f) : z;
    }
    bf16_t* y = (bf16_t*)p.y + (long)r * p.ldy + cb;
    const uint4 hi = pack8(x);
    *(uint4*)y = hi;
    if (p.y_split) {  // [hi | lo | hi]: lo = bf16(z - hi), exact in fp32
      float h[8], lo[8];
      unpack8(hi, h);
#pragma unroll
      for (int i = 0; i < 8; ++i) lo[i] = x[i] - h[i];
      *(uint4*)(y + p.c) = pack8(lo);
      *(uint4*)(y + 2 * p.c) = hi;
    }
  }
}

// backward reduction: g = dy * relu'(z) (z recomputed from x and the saved statistics);
// sums of g and g * xhat per channel -> dbeta, dgamma (+=) and the apply constants
template <bool F32>
__global__ __launch_bounds__(BN_T) void bn_bwd_reduce_kernel(const EncdiffBatchNormArgs p) {
  const BnLayout L(p.c);
  const bf16_t* DY = (const bf16_t*)p.dy;
  const int per = (p.rows + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * per, r1 = min(p.rows, r0 + per);
  float q[2][8], m[8], rs[8], ga[8], be[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) q[0][i] = q[1][i] = 0.f;
  if (L.pl < L.lanes) {
    const int cb = L.v * 8;
    ld8f(p.mean + cb, m);
    ld8f(p.rstd + cb, rs);
    ld8f(p.gamma + cb, ga);
    ld8f(p.beta + cb, be);
#pragma unroll 8
    for (int r = r0 + L.pl; r < r1; r += L.lanes) {
      float x[8], d[8];
      ld_x8<F32>(p.x, (long)r * p.ldx + cb, x);
      unpack8(*(const uint4*)(DY + (long)r * p.lddy + cb), d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (x[i] - m[i]) * rs[i];
        const float g = (p.relu && xh * ga[i] + be[i] <= 0.f) ? 0.f : d[i];
        q[0][i] += g;
        q[1][i] += g * xh;
      }
    }
  }
  float* part = p.partials + (long)blockIdx.x * 2 * p.c;
  bn_block_partial<2>(q, L, p.c, part);
  if (!bn_last_block(p.counter)) return;
  float* coef = p.partials + (long)gridDim.x * 2 * p.c;  // [2][c]: mean(g), mean(g * xhat)
  __shared__ double tot[2 * BN_T];
  bn_fold(p.partials, gridDim.x, p.c, tot);
  for (int ch = threadIdx.x; ch < p.c; ch += BN_T) {
    const double s = tot[ch], sx = tot[p.c + ch];
    p.dbeta[ch] += (float)s;
    p.dgamma[ch] += (float)sx;
    coef[ch] = (float)(s / p.rows);
    coef[p.c + ch] = (float)(sx / p.rows);
  }
  if (threadIdx.x == 0) *p.counter = 0u;
}

// dx = gamma * rstd * (g - mean(g) - xhat * mean(g * xhat))
template <bool F32>
__global__ __launch_bounds__(BN_T) void bn_bwd_apply_kernel(const EncdiffBatchNormArgs p, int nblk_reduce) {
  const int nv = p.c >> 3;
  const int total = p.rows * nv;  // < 2^31 (bn_check): 32-bit index math
  const float* coef = p.partials + (long)nblk_reduce * 2 * p.c;
  for (int e = blockIdx.x * BN_T + threadIdx.x; e < total; e += gridDim.x * BN_T) {
    const int r = e / nv;
    const int cb = (e - r * nv) * 8;
    float x[8], d[8], m[8], rs[8], ga[8], be[8], c0[8], c1[8];
    ld_x8<F32>(p.x, (long)r * p.ldx + cb, x);
    unpack8(*(const uint4*)((const bf16_t*)p.dy + r * p.lddy + cb), d);
    ld8f(p.mean + cb, m);
    ld8f(p.rstd + cb, rs);
    ld8f(p.gamma + cb, ga);
    ld8f(p.beta + cb, be);
    ld8f(coef + cb, c0);
    ld8f(coef + p.c + cb, c1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xh = (x[i] - m[i]) * rs[i];
      const float g = (p.relu && xh * ga[i] + be[i] <= 0.f) ? 0.f : d[i];
      x[i] = ga[i] * rs[i] * (g - c0[i] - xh * c1[i]);
    }
    *(uint4*)((bf16_t*)p.dx + r * p.lddx + cb) = pack8(x);
  }
}

// fp32 NCHW [B][C][H][W] -> bf16 [B*H*W][ld] with channels [C, cpad) zero; split: the row is
// the split-bf16 blocks [hi | lo | hi] of cpad channels each
__global__ __launch_bounds__(256) void nchw_to_rows_kernel(const float* __restrict__ x, int B, int C, int HW,
                                                           int cpad, bf16_t* __restrict__ y, long ld, int split) {
  const long total = (long)B * HW;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < total; i += (long)gridDim.x * 256) {
    const long b = i / HW, px = i - b * HW;
    for (int c0 = 0; c0 < cpad; c0 += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (c0 + k < C) ? x[(b * C + c0 + k) * HW + px] : 0.f;
      const uint4 hi = pack8(v);
      *(uint4*)(y + i * ld + c0) = hi;
      if (split) {
        float h[8];
        unpack8(hi, h);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] -= h[k];
        *(uint4*)(y + i * ld + cpad + c0) = pack8(v);
        *(uint4*)(y + i * ld + 2 * cpad + c0) = hi;
      }
    }
  }
}

int bn_check(const EncdiffBatchNormArgs* a) {
  if (!a || !a->x || !a->mean || !a->rstd || !a->gamma || !a->beta || !a->partials || !a->counter)
    return ENCDIFF_ERR_ARG;
  // 8-channel vectors must tile the 256 threads; the fold needs c <= 256
  if (a->rows <= 0 || a->c <= 0 || a->c % 8 || a->c > 256 || BN_T % (a->c / 8) || BN_T % a->c)
    return ENCDIFF_ERR_SHAPE;
  if (a->ldx % 8) return ENCDIFF_ERR_SHAPE;
  if (a->x_f32 && ((uintptr_t)a->x % 16)) return ENCDIFF_ERR_ARG;  // float4 loads
  if ((long)a->rows * (a->c / 8) >= (1L << 31)) return ENCDIFF_ERR_SHAPE;  // 32-bit apply indices
  for (const void* q : {(const void*)a->mean, (const void*)a->rstd, (const void*)a->gamma, (const void*)a->beta,
                        (const void*)a->partials})
    if ((uintptr_t)q % 16) return ENCDIFF_ERR_ARG;  // ld8f's 16-byte loads
  return ENCDIFF_OK;
}

int apply_grid(const EncdiffBatchNormArgs* a) {
  long g = ((long)a->rows * (a->c / 8) + BN_T - 1) / BN_T;
  return (int)(g > 4096 ? 4096 : g);
}

}  // namespace

extern "C" int encdiff_batchnorm_partials_floats(int rows, int c) {
  return bn_blocks(rows) * 2 * c + 2 * c;
}

extern "C" int encdiff_batchnorm_fwd(const EncdiffBatchNormArgs* a, void* stream) {
  const int rc = bn_check(a);
  if (rc) return rc;
  if (!a->y || a->ldy % 8 || (a->y_split && a->ldy < 3L * a->c)) return ENCDIFF_ERR_ARG;
  if (a->running_mean && !a->running_var) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = bn_blocks(a->rows);
  if (a->x_f32) hipLaunchKernelGGL(bn_stats_kernel<true>, dim3(nblk), dim3(BN_T), 0, s, *a);
  else hipLaunchKernelGGL(bn_stats_kernel<false>, dim3(nblk), dim3(BN_T), 0, s, *a);
  ED_CHECK_LAUNCH();
  if (a->x_f32) hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(apply_grid(a)), dim3(BN_T), 0, s, *a);
  else hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(apply_grid(a)), dim3(BN_T), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_batchnorm_apply(const EncdiffBatchNormArgs* a, void* stream) {
  // eval-mode BatchNorm (+ReLU): y = (x - mean) * rstd * gamma + beta with the caller's mean /
  // rstd (running statistics); partials / counter unused
  if (!a || !a->x || !a->y || !a->mean || !a->rstd || !a->gamma || !a->beta) return ENCDIFF_ERR_ARG;
  if (a->rows <= 0 || a->c <= 0 || a->c % 8 || a->ldx % 8 || a->ldy % 8) return ENCDIFF_ERR_SHAPE;
  if (a->y_split && a->ldy < 3L * a->c) return ENCDIFF_ERR_ARG;
  if ((long)a->rows * (a->c / 8) >= (1L << 31)) return ENCDIFF_ERR_SHAPE;
  for (const void* q : {(const void*)a->mean, (const void*)a->rstd, (const void*)a->gamma, (const void*)a->beta})
    if ((uintptr_t)q % 16) return ENCDIFF_ERR_ARG;
  if (a->x_f32 && ((uintptr_t)a->x % 16)) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (a->x_f32) hipLaunchKernelGGL(bn_apply_kernel<true>, dim3(apply_grid(a)), dim3(BN_T), 0, s, *a);
  else hipLaunchKernelGGL(bn_apply_kernel<false>, dim3(apply_grid(a)), dim3(BN_T), 0, s, *a);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_batchnorm_bwd(const EncdiffBatchNormArgs* a, void* stream) {
  const int rc = bn_check(a);
  if (rc) return rc;
  if (!a->dy || !a->dx || !a->dgamma || !a->dbeta || a->lddy % 8 || a->lddx % 8) return ENCDIFF_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = bn_blocks(a->rows);
  if (a->x_f32) hipLaunchKernelGGL(bn_bwd_reduce_kernel<true>, dim3(nblk), dim3(BN_T), 0, s, *a);
  else hipLaunchKernelGGL(bn_bwd_reduce_kernel<false>, dim3(nblk), dim3(BN_T), 0, s, *a);
  ED_CHECK_LAUNCH();
  if (a->x_f32) hipLaunchKernelGGL(bn_bwd_apply_kernel<true>, dim3(apply_grid(a)), dim3(BN_T), 0, s, *a, nblk);
  else hipLaunchKernelGGL(bn_bwd_apply_kernel<false>, dim3(apply_grid(a)), dim3(BN_T), 0, s, *a, nblk);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

static int nchw_to_rows(const float* x, int batch, int c, int hw, int cpad, void* y, long ldy, int split,
                        void* stream) {
  if (!x || !y || batch <= 0 || c <= 0 || hw <= 0 || cpad < c || cpad % 8 || ldy < (split ? 3 : 1) * cpad || ldy % 8)
    return ENCDIFF_ERR_ARG;
  long g = ((long)batch * hw + 255) / 256;
  hipLaunchKernelGGL(nchw_to_rows_kernel, dim3((unsigned)(g > 4096 ? 4096 : g)), dim3(256), 0, (hipStream_t)stream,
                     x, batch, c, hw, cpad, (bf16_t*)y, ldy, split);
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}

extern "C" int encdiff_nchw_to_rows(const float* x, int batch, int c, int hw, int cpad, void* y, long ldy,
                                    void* stream) {
  return nchw_to_rows(x, batch, c, hw, cpad, y, ldy, 0, stream);
}

extern "C" int encdiff_nchw_to_rows_split3(const float* x, int batch, int c, int hw, int cpad, void* y, long ldy,
                                           void* stream) {
  return nchw_to_rows(x, batch, c, hw, cpad, y, ldy, 1, stream);
}
