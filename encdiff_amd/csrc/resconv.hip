// resconv.hip -- an inference ResBlock convolution with its GroupNorm, one launch
// (include/encdiff_hip.h EncdiffResConvArgs; openaimodel_enc.py:255-275).
//
// At sampling batches (DDIM, B = 8) every ResBlock of the unfused path is four to five launches
// of a few microseconds each -- GroupNorm, conv, GroupNorm(+FiLM), conv, skip / resample -- that
// each sit at the launch-and-load-latency floor, not at a bandwidth or MFMA bound.  Here a
// workgroup owns (a slice of 16 * TN output channels, a chunk of 16-row output tiles of one image
// group) and
//   1. stages the WHOLE images of its group into LDS (row stride cin + 8 elements: the 16 rows of
//      an MFMA fragment read hit distinct banks) and reduces their per-(image, group) statistics
//      from that one pass -- one image per group above 4x4, four 2x2 images per 16-row tile;
//   2. normalises the staged rows in place (GroupNorm (+FiLM) (+SiLU), rounded to bf16 as the
//      GroupNorm launch stores them), DOWN2: avg-pools them into a second region;
//   3. runs the implicit im2col GEMM: A fragments gathered from LDS per tap (zero padding at the
//      conv resolution, UP2 through the parent pixel), B fragments streamed from L2 in batches
//      of 8 k-steps, double-buffered; the 4 waves split the chunk's tiles and, when the chunk has
//      fewer than 4 tiles, the k range (partials added in wave order through LDS);
//   4. adds bias, the 1x1 skip conv (its own k loop, rounded to bf16 as the skip launch stores
//      it) or the (resampled) residual rows, and stores bf16.
// The redundant per-workgroup statistics (every slice workgroup of an image re-reduces it) cost
// L2 reads of at most ~100 KB per workgroup -- far below the launches they replace.
#include "common.h"

namespace {

#ifndef RC_NT
#define RC_NT 512  // threads per workgroup (256: 648 us per UNet forward of fused convs at B = 8, 512: 617, 1024: spills)
#endif
constexpr int RC_THREADS = RC_NT;
constexpr int RC_NW = RC_NT / 64;  // waves per workgroup
constexpr int RC_PAD = 8;   // LDS row padding (bf16 elements)
constexpr int RC_D = 8;     // k-steps per B prefetch batch
constexpr int RC_LDS_MAX = 160 * 1024;
constexpr int RC_CE = 8;    // (image, channel) coefficient entries per thread (host: ipw * cin <= 2048)
ED_DEV void load8f_(const float* p, float* v) {  // (no alignment assumed: parameter views)
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = p[i];
}
#ifndef RC_U
#define RC_U 16  // staging rows in flight per thread
#endif

#ifndef RC_STAMP
#define RC_STAMP 0  // diagnostic builds: phase stamps (tools/rc_stamps.py)
#endif
// v + v of lane ^ 16 / ^ 32 (gfx950 permlane swaps: VALU, no LDS round trip)
ED_DEV float rc_sum_x16(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
ED_DEV float rc_sum_x32(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

#if RC_STAMP
// per workgroup, thread 0: [0] realtime at entry, [1..8] shader clock at entry / operands issued /
// staged / statistics / window normalised (B landed) / GEMM done / k-split combined / exit,
// [9] realtime at exit
__device__ unsigned long long rc_stamps[4096][10];
// per wave (lane 0): [w][0] entry, [w][1] operands issued, [w][2] staged (own loads landed),
// [w][3] arrival at the statistics barrier
__device__ unsigned long long rc_wstamps[4096][16][4];
#define RC_WST(i)                                                                                    \
  do {                                                                                               \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) rc_wstamps[blockIdx.x][threadIdx.x >> 6][i] = __builtin_readcyclecounter(); \
  } while (0)
#define RC_ST(i)                                                                                     \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 4096) rc_stamps[blockIdx.x][i] = __builtin_readcyclecounter(); \
  } while (0)
#define RC_ST_RT(i)                                                                                  \
  do {                                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 4096) rc_stamps[blockIdx.x][i] = wall_clock64();           \
  } while (0)
#else
#define RC_ST(i) do {} while (0)
#define RC_ST_RT(i) do {} while (0)
#define RC_WST(i) do {} while (0)
#endif

struct RcPlan {
  int ho, hwo, ipw;         // conv (output) resolution, its pixels per image, images per group
  int mc, wk;               // 16-row tiles per workgroup (= waves along M), k-split (mc * wk == RC_NW)
  int nchunk, ngroup;       // tile chunks per group, image groups
  int ldx;                  // LDS row stride (elements)
  int nsr, ncr;             // max staged rows per image (resolution h), max conv-input rows (DOWN2)
  int kl;                   // k-steps whose B fragments are staged in LDS (the rest stream from L2)
  int xs_off, ps_off, red_off, chs_off, gst_off, fl_off, zr_off, sk_off, bs_off, lds;
};

template <int TN>
__global__ __launch_bounds__(RC_THREADS) void resconv_kernel(const EncdiffResConvArgs p, const RcPlan q) {
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) const void gbl_void;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* xs = (bf16_t*)(smem + q.xs_off);    // [ipw][nsr * h][ldx] staged, then normalised rows
  bf16_t* ps = (bf16_t*)(smem + q.ps_off);    // DOWN2: [ipw][ncr * ho][ldx] pooled rows
  float* red = (float*)(smem + q.red_off);    // reduction partials, later the k-split partials
  float2* chs = (float2*)(smem + q.chs_off);  // [ipw][cin] channel sums (non-power-of-two nv)
  float2* gst = (float2*)(smem + q.gst_off);  // [ipw][groups] mean, rstd
  float* fl = (float*)(smem + q.fl_off);      // [ipw][2 cin] FiLM rows (scale | shift)
  bf16_t* zr = (bf16_t*)(smem + q.zr_off);    // a zero row: the gather's padding taps read it
  bf16_t* bs = (bf16_t*)(smem + q.bs_off);    // [kl][TN] B fragments, 1 KiB each, lane-linear
  bf16_t* sk = (bf16_t*)(smem + q.sk_off);    // skip conv: [mc][cskip/32] A, then [TN][cskip/32] B fragments
  RC_ST_RT(0);
  RC_ST(1);
  RC_WST(0);
  if (p.skip_stages & 128) return;  // timing experiments: the launch of this grid alone
  // the wave index as a scalar: everything derived from it (k ranges, taps, tile rows) stays in
  // SGPRs with scalar branches instead of exec-masked vector ones
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, g4 = lane >> 4;
  const int G = gridDim.x, bid = blockIdx.x;
  // XCD-aware order: consecutive logical indices run on one XCD (workgroup i -> XCD i % 8), and
  // the logical order is slice-major, so one XCD's L2 holds whole weight slices
  const int li = (G & 7) ? bid : (bid & 7) * (G >> 3) + (bid >> 3);
  const int per_slice = q.ngroup * q.nchunk;
  const int slice = li / per_slice, rem = li - slice * per_slice;
  const int grp = rem / q.nchunk, chunk = rem - grp * q.nchunk;
  const int cin = p.cin, nv = cin >> 3, h = p.h, hw = h * h, ipw = q.ipw;
  const int ho = q.ho, hwo = q.hwo;
  const int b0 = grp * ipw;
  const int n0 = slice * 16 * TN;
  const int spt = cin >> 5, KS = 9 * spt;  // k-steps per tap, in total
  const int KS2 = p.cskip >> 5;
  const int grow0 = b0 * hwo;  // first output row of the group
  const bool up = p.resample == ENCDIFF_RESAMPLE_UP2, down = p.resample == ENCDIFF_RESAMPLE_DOWN2;
  const int wm_i = wave % q.mc, wk_i = wave / q.mc;  // (wk_i < q.wk: mc * wk == RC_NW)
  const int mt = chunk * q.mc + wm_i;
  const int np = RC_THREADS / nv, tv = tid % nv, tp = tid / nv;
  const int cpg = cin / p.groups;

  // ---- 0. every global operand is requested up front, so the kernel waits for memory once:
  // B slice, skip-conv fragments and FiLM rows by LDS-DMA (one wave instruction per 1 KiB,
  // lane-linear), the affine parameters of this thread's channels and the epilogue's bias /
  // residual values into registers; the staging loads follow ----
  if (!(p.skip_stages & 20)) {
    for (int f = wave; f < q.kl * TN; f += RC_NW) {
      const int ks = f / TN, t = f - ks * TN;
      const bf16_t* src = (const bf16_t*)p.w + (long)(n0 + t * 16 + l16) * p.ld_w + ks * 32 + g4 * 8;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(bs + f * 512), 16, 0, 0);
    }
  }
  if (KS2) {
    for (int f = wave; f < (q.mc + TN) * KS2; f += RC_NW) {
      const int u = f / KS2, ks = f - u * KS2;
      const bf16_t* src = u < q.mc
          ? (const bf16_t*)p.xskip + (long)(grow0 + (chunk * q.mc + u) * 16 + l16) * p.ld_xskip + ks * 32 + g4 * 8
          : (const bf16_t*)p.wskip + (long)(n0 + (u - q.mc) * 16 + l16) * p.ld_wskip + ks * 32 + g4 * 8;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(sk + f * 512), 16, 0, 0);
    }
  }
  if (p.film) {  // (host: 16-byte aligned rows)
    const int n16 = cin >> 1;  // 16-byte chunks of one row
    for (int c = tid; c < ipw * n16; c += RC_THREADS) {
      const int jj = c / n16, o = c - jj * n16;
      __builtin_amdgcn_global_load_lds((gbl_void*)(p.film + (long)(b0 + jj) * p.ld_film + o * 4),
                                       (lds_void*)(fl + (c & ~63) * 4), 16, 0, 0);
    }
  }
  float ng[8], nb[8];  // GroupNorm affine of this thread's 8 channels
  load8f_(p.gamma + tv * 8, ng);
  load8f_(p.beta + tv * 8, nb);
  float eb[TN], esb[TN];  // epilogue: bias, skip bias; the residual as raw bf16 (converted last)
  bf16_t er[4][TN][4];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    eb[t] = esb[t] = 0.f;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
      for (int u = 0; u < 4; ++u) er[qq][t][u] = 0;
  }
  if (wk_i == 0) {
    const bf16_t* R = (const bf16_t*)p.resid;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int col = n0 + t * 16 + l16;
      if (p.bias) eb[t] = p.bias[col];
      if (KS2 && p.bskip) esb[t] = p.bskip[col];
      if (!R) continue;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int rr = mt * 16 + 4 * g4 + qq;
        const int jj = rr / hwo, pr = rr - jj * hwo, y = pr / ho, x = pr - y * ho;
        if (p.resid_resample == ENCDIFF_RESAMPLE_UP2) {
          const int hr = ho >> 1;
          er[qq][t][0] = R[((long)(b0 + jj) * hr * hr + (y >> 1) * hr + (x >> 1)) * p.ld_resid + col];
        } else if (p.resid_resample == ENCDIFF_RESAMPLE_DOWN2) {
          const int hr = ho << 1;
          const long r0 = (long)(b0 + jj) * hr * hr + 2 * y * hr + 2 * x;
          er[qq][t][0] = R[r0 * p.ld_resid + col];
          er[qq][t][1] = R[(r0 + 1) * p.ld_resid + col];
          er[qq][t][2] = R[(r0 + hr) * p.ld_resid + col];
          er[qq][t][3] = R[(r0 + hr + 1) * p.ld_resid + col];
        } else {
          er[qq][t][0] = R[(long)(grow0 + rr) * p.ld_resid + col];
        }
      }
    }
  }
  for (int i = tid; i < nv; i += RC_THREADS) *(uint4*)(zr + i * 8) = make_uint4(0u, 0u, 0u, 0u);
  RC_ST(2);
  RC_WST(1);

  // rows the workgroup's tiles read: conv-input rows [cy0, cy1] (resolution ho), staged rows
  // [sy0, sy1] (resolution h); whole images when a tile holds several
  int cy0 = 0, cy1 = ho - 1;
  if (ipw == 1) {
    const int r0 = chunk * q.mc * 16, r1 = r0 + q.mc * 16 - 1;
    cy0 = max(r0 / ho - 1, 0);
    cy1 = min(r1 / ho + 1, ho - 1);
  }
  const int sy0 = up ? cy0 >> 1 : (down ? 2 * cy0 : cy0);
  const int sy1 = up ? cy1 >> 1 : (down ? 2 * cy1 + 1 : cy1);
  const int px0 = sy0 * h, npx = (sy1 - sy0 + 1) * h;  // staged pixels of each image
  const int xis = q.nsr * h * q.ldx;                    // LDS image stride of xs

  // ---- 1. stage the window rows, per-channel sums over the WHOLE images ----
  const int lpi = np / ipw;  // pixel lanes per image (host: np >= ipw)
  const int j = tp / lpi, l = tp - j * lpi;
  float s[8], ss[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = ss[i] = 0.f;
  if (tp < lpi * ipw) {
    const bf16_t* src = (const bf16_t*)p.x + (long)(b0 + j) * hw * p.ld_x + tv * 8;
    bf16_t* dst = xs + j * xis + tv * 8 - px0 * q.ldx;
    auto acc = [&](const uint4& u, int px) {
      if ((unsigned)(px - px0) < (unsigned)npx) *(uint4*)(dst + px * q.ldx) = u;
      float v[8];
      unpack8(u, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] += v[i]; ss[i] += v[i] * v[i]; }
    };
    int px = l;
    if (!(p.skip_stages & 1)) {
      // RC_U rows in flight per thread: the staging is one or two load round trips (a 96 KB image
      // at 16x16 x 192 channels is 26 rows per thread)
      for (; px + (RC_U - 1) * lpi < hw; px += RC_U * lpi) {
        uint4 u[RC_U];
#pragma unroll
        for (int r = 0; r < RC_U; ++r) u[r] = *(const uint4*)(src + (long)(px + r * lpi) * p.ld_x);
#pragma unroll
        for (int r = 0; r < RC_U; ++r) acc(u[r], px + r * lpi);
      }
      for (; px < hw; px += lpi) acc(*(const uint4*)(src + (long)px * p.ld_x), px);
    }
  }
  // every operand this wave requested has landed (loads return in order: the staging loads were
  // the last); the barrier below publishes all waves' LDS-DMA with the staged rows
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  RC_ST(3);
  RC_WST(2);
  if (p.skip_stages & 256) return;  // timing experiments: launch + the prologue's memory round trip

  // ---- statistics.  Power-of-two nv: xor-shuffles over the lanes of one image inside a wave
  // (lane offsets nv, 2 nv, ...), the owner lane folds its 8 channels into group partials (or
  // keeps the vector's partial when a group spans vectors), at most 4 wave rows per image meet in
  // LDS.  Otherwise every lane row goes through LDS per channel, then per group. ----
  const bool pow2 = (nv & (nv - 1)) == 0;
  const float inv_n = 1.f / ((float)hw * (float)cpg);
  if (pow2) {
    const int span = min(64, lpi * nv);  // lanes of one image inside a wave
    // lane offsets 16 / 32 by the gfx950 permlane swaps (VALU; a + b in either order: the same bits
    // as the ds_bpermute shuffle), 4 / 8 by shuffles -- 16 serial LDS round trips per wave were
    // ~3 000 cycles before the first barrier (per-wave stamps, tools/rc_stamps.py --waves)
#pragma unroll
    for (int o = 4; o < 16; o <<= 1) {
      if (o < nv || o >= span) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] += __shfl_xor(s[i], o, 64);
        ss[i] += __shfl_xor(ss[i], o, 64);
      }
    }
    if (16 >= nv && 16 < span) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] = rc_sum_x16(s[i]); ss[i] = rc_sum_x16(ss[i]); }
    }
    if (32 >= nv && 32 < span) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { s[i] = rc_sum_x32(s[i]); ss[i] = rc_sum_x32(ss[i]); }
    }
    const int nr = lpi * nv >= 64 ? lpi * nv / 64 : 1;  // partial rows per image
    const int nslot = cpg <= 8 ? p.groups : nv;        // slots per row: groups, or vectors
    if ((lane & (span - 1)) < nv) {
      const int r = lpi * nv >= 64 ? wave - j * nr : 0;
      float2* row = (float2*)red + (j * nr + r) * nslot;
      if (cpg <= 8) {
        for (int k = 0; k < 8 / cpg; ++k) {
          float a = 0.f, b = 0.f;
          for (int i = k * cpg; i < (k + 1) * cpg; ++i) { a += s[i]; b += ss[i]; }
          row[tv * (8 / cpg) + k] = make_float2(a, b);
        }
      } else {
        float a = 0.f, b = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) { a += s[i]; b += ss[i]; }
        row[tv] = make_float2(a, b);
      }
    }
    RC_WST(3);
    __syncthreads();
    for (int e = tid; e < ipw * p.groups; e += RC_THREADS) {  // (image, group): rows, then vectors in order
      const int jj = e / p.groups, g = e - jj * p.groups;
      const int vpg = cpg <= 8 ? 1 : cpg / 8, s0 = cpg <= 8 ? g : g * vpg;
      float a = 0.f, b = 0.f;
      for (int r = 0; r < nr; ++r)
        for (int v = 0; v < vpg; ++v) {
          const float2 t = ((const float2*)red)[(jj * nr + r) * nslot + s0 + v];
          a += t.x;
          b += t.y;
        }
      const float mean = a * inv_n;
      const float var = fmaxf(b * inv_n - mean * mean, 0.f);
      gst[e] = make_float2(mean, rsqrtf(var + p.eps));
    }
  } else {  // (host: one image per group) lanes l, l + nv, l + 2 nv of a wave share a channel vector
    float* rs = red + wave * cin;
    float* rq = red + (RC_NW + wave) * cin;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float a = s[i], b = ss[i];
      for (int k = 1; k * nv < 64; ++k) {
        const int src = lane + k * nv;
        const float ta = __shfl(s[i], src < 64 ? src : lane, 64), tb = __shfl(ss[i], src < 64 ? src : lane, 64);
        if (src < 64) { a += ta; b += tb; }
      }
      s[i] = a;
      ss[i] = b;
    }
    if (lane < nv) {  // the wave's first nv lanes cover every channel vector once (zeros past np)
      const int c0 = ((wave * 64 + lane) % nv) * 8;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        rs[c0 + i] = s[i];
        rq[c0 + i] = ss[i];
      }
    }
    __syncthreads();
    for (int e = tid; e < cin; e += RC_THREADS) {  // channel: the waves' rows in order
      float a = 0.f, b = 0.f;
#pragma unroll 4
      for (int r = 0; r < RC_NW; ++r) { a += red[r * cin + e]; b += red[(RC_NW + r) * cin + e]; }
      chs[e] = make_float2(a, b);
    }
    __syncthreads();
    for (int e = tid; e < ipw * p.groups; e += RC_THREADS) {  // (image, group)
      const int jj = e / p.groups, g = e - jj * p.groups;
      float a = 0.f, b = 0.f;
#pragma unroll 4
      for (int c = g * cpg; c < (g + 1) * cpg; ++c) { const float2 v = chs[jj * cin + c]; a += v.x; b += v.y; }
      const float mean = a * inv_n;
      const float var = fmaxf(b * inv_n - mean * mean, 0.f);
      gst[e] = make_float2(mean, rsqrtf(var + p.eps));
    }
  }
  __syncthreads();
  RC_ST(4);

  // ---- 2. normalise the window in place (bf16, as the GroupNorm launch stores it): a thread's
  // 8 channels' coefficients from the group statistics, its affine registers and the FiLM rows;
  // DOWN2: pool into ps ----
  const int ncr = cy1 - cy0 + 1, pis = q.ncr * ho * q.ldx;
  if (!(p.skip_stages & 2)) {
    const bool silu = p.silu;
    if (tp < lpi * ipw) {  // thread = (image j, channel vector tv, pixel lane l), as in the staging
      float mul[8], add[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // y = ((x - m) r ga + be)(1 + sc) + sh
        const float2 st = gst[j * p.groups + (tv * 8 + i) / cpg];
        float a = st.y * ng[i], bb = nb[i] - st.x * a;
        if (p.film) {
          const float sc = fl[j * 2 * cin + tv * 8 + i], sf = fl[j * 2 * cin + cin + tv * 8 + i];
          a *= (1.f + sc);
          bb = bb * (1.f + sc) + sf;
        }
        mul[i] = a;
        add[i] = bb;
      }
      bf16_t* base = xs + j * xis + tv * 8;
      for (int pl = l; pl < npx; pl += 4 * lpi) {  // four rows' reads issued before any math
        uint4 u[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
          if (pl + d * lpi < npx) u[d] = *(const uint4*)(base + (pl + d * lpi) * q.ldx);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          if (pl + d * lpi < npx) {
            float v[8];
            unpack8(u[d], v);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              const float z = v[i] * mul[i] + add[i];
              v[i] = silu ? silu_f(z) : z;
            }
            *(uint4*)(base + (pl + d * lpi) * q.ldx) = pack8(v);
          }
        }
      }
    }
    if (down) {  // ew_kernel RESAMPLE's order: ((a + b) + c + d) / 4, rounded to bf16
      __syncthreads();
      for (int e = tid; e < ipw * ncr * ho * nv; e += RC_THREADS) {
        const int px = e / nv, cv = e - px * nv, jj = px / (ncr * ho), pr = px - jj * ncr * ho;
        const int y = pr / ho, x = pr - y * ho;  // pooled row cy0 + y <- staged rows 2 y, 2 y + 1
        const bf16_t* s0 = xs + jj * xis + (2 * y * h + 2 * x) * q.ldx + cv * 8;
        float o[8], t[8];
        unpack8(*(const uint4*)s0, o);
        unpack8(*(const uint4*)(s0 + q.ldx), t);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += t[i];
        unpack8(*(const uint4*)(s0 + h * q.ldx), t);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += t[i];
        unpack8(*(const uint4*)(s0 + (h + 1) * q.ldx), t);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (o[i] + t[i]) * 0.25f;
        *(uint4*)(ps + jj * pis + (y * ho + x) * q.ldx + cv * 8) = pack8(o);
      }
    }
  }
  __syncthreads();
  RC_ST(5);

  // ---- 3. implicit-im2col GEMM: this wave's 16-row tile x TN column tiles over its k range ----
  const int ra = mt * 16 + l16;  // group row of this lane's A row
  const int ja = ra / hwo, pa = ra - ja * hwo, oy = pa / ho, ox = pa - oy * ho;
  // gather region: conv-input rows from gy0 (its own resolution), width gw, UP2 through >> 1;
  // a padding tap reads the zero row (no divergent branch around the fragment read)
  const bf16_t* gbase = (down ? ps + ja * pis : xs + ja * xis) + g4 * 8;
  const int gy0 = down ? cy0 : sy0, gw = down ? ho : h, us = up ? 1 : 0;
  const int per = ((KS + q.wk - 1) / q.wk + 1) & ~1, k0 = min(KS, wk_i * per), k1 = min(KS, k0 + per);
  const int kl = min(k1, q.kl);
  v4f acc[TN], acc2[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) acc[t] = acc2[t] = (v4f){0.f, 0.f, 0.f, 0.f};
  auto apix = [&](int tap) -> const bf16_t* {
    const int ty = tap / 3;
    const int sy = oy + ty - 1, sx = ox + (tap - 3 * ty) - 1;
    const bool ok = (unsigned)sy < (unsigned)ho && (unsigned)sx < (unsigned)ho;
    return ok ? gbase + (((sy >> us) - gy0) * gw + (sx >> us)) * q.ldx : zr + g4 * 8;
  };
  if (!(p.skip_stages & 36) && k0 < kl) {
    // B from LDS, four k-steps per iteration with all their fragment reads issued first; the tap
    // (and with it the A pixel address) advances by a uniform branch
    int tap = k0 / spt, cc = k0 - tap * spt;
    const bf16_t* ap = apix(tap);
    for (int s0 = k0; s0 < kl; s0 += 4) {
      const bf16_t* aq[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        aq[d] = ap + cc * 32;
        if (++cc == spt) {
          cc = 0;
          ap = apix(++tap);
        }
      }
      v8bf a[4], b[4][TN];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int ks = min(s0 + d, kl - 1);
        a[d] = *(const v8bf*)aq[d];
#pragma unroll
        for (int t = 0; t < TN; ++t) b[d][t] = *(const v8bf*)(bs + ((ks * TN + t) * 64 + lane) * 8);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if (s0 + d < kl) {
#pragma unroll
          for (int t = 0; t < TN; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[d], b[d][t], acc[t], 0, 0, 0);
        }
      }
    }
  }
  // k-steps past the LDS budget: B streamed from L2 in double-buffered batches of RC_D.  Always
  // issued (a step past the range re-loads the last one) so the loads are straight-line code the
  // compiler counts (vmcnt) instead of draining per batch.
  const int kt0 = max(k0, kl);
  const bf16_t* wp = (const bf16_t*)p.w + (long)(n0 + l16) * p.ld_w + g4 * 8;
  auto loadb = [&](v8bf (&b)[RC_D][TN], int s0) {
#pragma unroll
    for (int d = 0; d < RC_D; ++d) {
      const int ks = min(s0 + d, k1 - 1);
#pragma unroll
      for (int t = 0; t < TN; ++t) b[d][t] = *(const v8bf*)(wp + (long)t * 16 * p.ld_w + ks * 32);
    }
  };
  auto compute = [&](const v8bf (&b)[RC_D][TN], int s0) {
#pragma unroll
    for (int d = 0; d < RC_D; ++d) {
      if (s0 + d < k1) {
        const int ks = s0 + d, tap = ks / spt;
        const v8bf a = *(const v8bf*)(apix(tap) + (ks - tap * spt) * 32);
#pragma unroll
        for (int t = 0; t < TN; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[d][t], acc[t], 0, 0, 0);
      }
    }
  };
  if (kt0 < k1 && !(p.skip_stages & 36)) {
    v8bf b0q[RC_D][TN], b1q[RC_D][TN];
    loadb(b0q, kt0);
    for (int s0 = kt0; s0 < k1; s0 += 2 * RC_D) {
      loadb(b1q, s0 + RC_D);
      compute(b0q, s0);
      if (s0 + 2 * RC_D < k1) loadb(b0q, s0 + 2 * RC_D);
      compute(b1q, s0 + RC_D);
    }
  }
  // 1x1 skip conv from its LDS fragments (its own accumulator: rounded to bf16 with its bias, as
  // the skip launch stores it)
  if (KS2) {
    const int per2 = (KS2 + q.wk - 1) / q.wk, j0 = wk_i * per2, j1 = min(KS2, j0 + per2);
    for (int ks = j0; ks < j1; ++ks) {
      const v8bf a = *(const v8bf*)(sk + ((wm_i * KS2 + ks) * 64 + lane) * 8);
#pragma unroll
      for (int t = 0; t < TN; ++t)
        acc2[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
            a, *(const v8bf*)(sk + (((q.mc + t) * KS2 + ks) * 64 + lane) * 8), acc2[t], 0, 0, 0);
    }
  }
  RC_ST(6);
  // k-split partials: waves 1.. of a tile hand theirs to wave 0 through LDS (added in wave order)
  if (q.wk > 1) {
    float* wr = red + ((wk_i - 1) * q.mc + wm_i) * (2 * TN * 256);
    if (wk_i > 0) {
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        *(v4f*)(wr + (t * 64 + lane) * 4) = acc[t];
        *(v4f*)(wr + ((TN + t) * 64 + lane) * 4) = acc2[t];
      }
    }
    __syncthreads();
    if (wk_i > 0) return;
    for (int w = 1; w < q.wk; ++w) {
      const float* o = red + ((w - 1) * q.mc + wm_i) * (2 * TN * 256);
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        acc[t] += *(const v4f*)(o + (t * 64 + lane) * 4);
        acc2[t] += *(const v4f*)(o + ((TN + t) * 64 + lane) * 4);
      }
    }
  }
  RC_ST(7);
  // ---- 4. epilogue: bias, skip / residual (prefetched), bf16 store ----
  bf16_t* Y = (bf16_t*)p.y;
#pragma unroll
  for (int qq = 0; qq < 4; ++qq) {
    const long grow = grow0 + mt * 16 + 4 * g4 + qq;  // accumulator element qq: row 4 g4 + qq, column l16
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      float v = acc[t][qq] + eb[t];
      if (KS2) v += bf16_round(acc2[t][qq] + esb[t]);
      if (p.resid_resample == ENCDIFF_RESAMPLE_DOWN2) {  // ew_kernel RESAMPLE's order, rounded to bf16
        float o = bf2f(er[qq][t][0]) + bf2f(er[qq][t][1]);
        o += bf2f(er[qq][t][2]);
        v += bf16_round((o + bf2f(er[qq][t][3])) * 0.25f);
      } else {
        v += bf2f(er[qq][t][0]);
      }
      if (!(p.skip_stages & 8)) Y[grow * p.ld_y + n0 + t * 16 + l16] = f2bf(v);
    }
  }
  RC_ST(8);
  RC_ST_RT(9);
}

int rc_plan(const EncdiffResConvArgs& a, RcPlan& q, int& tn) {
  if (!a.x || !a.w || !a.y || !a.gamma || !a.beta) return ENCDIFF_ERR_ARG;
  if (a.batch <= 0 || a.h <= 0 || a.cin % 32 || a.cout % 16 || a.groups <= 0 || a.cin % a.groups) return ENCDIFF_ERR_SHAPE;
  if (a.ld_x % 8 || a.ld_w % 8 || a.ld_x < a.cin || a.ld_w < 9 * a.cin || a.ld_y < a.cout) return ENCDIFF_ERR_SHAPE;
  if (a.cin > 512 || a.groups > 64) return ENCDIFF_ERR_UNSUPPORTED;
  if (a.film && (((uintptr_t)a.film & 15) || a.ld_film % 4)) return ENCDIFF_ERR_UNSUPPORTED;  // LDS-DMA rows
  if (a.resample < 0 || a.resample > 2 || a.resid_resample < 0 || a.resid_resample > 2) return ENCDIFF_ERR_ARG;
  if (a.resample == ENCDIFF_RESAMPLE_DOWN2 && a.h % 2) return ENCDIFF_ERR_SHAPE;
  if (a.cskip && (!a.xskip || !a.wskip || a.cskip % 32 || a.ld_xskip % 8 || a.ld_wskip % 8 || a.resid))
    return ENCDIFF_ERR_ARG;
  q.ho = a.resample == ENCDIFF_RESAMPLE_UP2 ? 2 * a.h : a.resample == ENCDIFF_RESAMPLE_DOWN2 ? a.h / 2 : a.h;
  q.hwo = q.ho * q.ho;
  if (a.resid_resample == ENCDIFF_RESAMPLE_UP2 && q.ho % 2) return ENCDIFF_ERR_SHAPE;
  if (q.hwo < 16 && 16 % q.hwo) return ENCDIFF_ERR_UNSUPPORTED;
  if (q.hwo >= 16 && q.hwo % 16) return ENCDIFF_ERR_UNSUPPORTED;
  q.ipw = q.hwo >= 16 ? 1 : 16 / q.hwo;
  if (a.batch % q.ipw) return ENCDIFF_ERR_UNSUPPORTED;
  const int nv = a.cin / 8, np = RC_THREADS / nv;
  if (np < q.ipw || q.ipw * a.cin > RC_CE * RC_THREADS) return ENCDIFF_ERR_UNSUPPORTED;
  if ((nv & (nv - 1)) && q.ipw != 1) return ENCDIFF_ERR_UNSUPPORTED;  // non-power-of-two statistics path
  tn = a.tile_n ? a.tile_n : 1;
  if ((tn != 1 && tn != 2) || a.cout % (16 * tn)) return ENCDIFF_ERR_ARG;
  const int mtg = q.ipw * q.hwo / 16, nslice = a.cout / (16 * tn);
  q.ngroup = a.batch / q.ipw;
  if (a.tile_m) {
    if ((a.tile_m != 1 && a.tile_m != 2 && a.tile_m != 4) || mtg % a.tile_m) return ENCDIFF_ERR_ARG;
    q.mc = a.tile_m;
  } else {  // up to 4 tiles per workgroup, fewer while that leaves < 256 workgroups (tools/rc_bench.py
            // --tiles at B = 8: 16x16 x 64 channels 11.6 -> 10.8 us with 2 tiles / 256 workgroups)
    q.mc = mtg >= 4 ? 4 : mtg >= 2 ? 2 : 1;
    while (q.mc > 1 && q.ngroup * (mtg / q.mc) * nslice < 256) q.mc >>= 1;
  }
  q.wk = RC_NW / q.mc;
  q.nchunk = mtg / q.mc;
  q.ldx = a.cin + RC_PAD;
  // the largest row window of any chunk (kernel: cy0 / cy1 / sy0 / sy1)
  q.nsr = q.ncr = 0;
  for (int c = 0; c < q.nchunk; ++c) {
    int cy0 = 0, cy1 = q.ho - 1;
    if (q.ipw == 1) {
      const int r0 = c * q.mc * 16, r1 = r0 + q.mc * 16 - 1;
      cy0 = r0 / q.ho - 1 > 0 ? r0 / q.ho - 1 : 0;
      cy1 = r1 / q.ho + 1 < q.ho - 1 ? r1 / q.ho + 1 : q.ho - 1;
    }
    const bool up = a.resample == ENCDIFF_RESAMPLE_UP2, down = a.resample == ENCDIFF_RESAMPLE_DOWN2;
    const int sy0 = up ? cy0 >> 1 : (down ? 2 * cy0 : cy0), sy1 = up ? cy1 >> 1 : (down ? 2 * cy1 + 1 : cy1);
    if (sy1 - sy0 + 1 > q.nsr) q.nsr = sy1 - sy0 + 1;
    if (cy1 - cy0 + 1 > q.ncr) q.ncr = cy1 - cy0 + 1;
  }
  int off = 0;
  auto take = [&](long bytes) { const int o = off; off += (int)((bytes + 15) & ~15L); return o; };
  q.xs_off = take((long)q.ipw * q.nsr * a.h * q.ldx * 2);
  q.ps_off = a.resample == ENCDIFF_RESAMPLE_DOWN2 ? take((long)q.ipw * q.ncr * q.ho * q.ldx * 2) : q.xs_off;
  const long red_f = (nv & (nv - 1)) ? 2L * RC_NW * a.cin : 2L * 16 * 64, kred_f = (q.wk - 1L) * q.mc * 2 * tn * 256;
  q.red_off = take(4 * (red_f > kred_f ? red_f : kred_f));
  q.chs_off = take((nv & (nv - 1)) ? 8L * q.ipw * a.cin : 0);
  q.gst_off = take(8L * q.ipw * a.groups);
  q.fl_off = take(a.film ? 8L * q.ipw * a.cin : 0);
  q.zr_off = take(2L * a.cin);
  q.sk_off = take((long)(q.mc + tn) * (a.cskip / 32) * 1024);
  q.bs_off = off;
  const int ks = 9 * a.cin / 32, room = (RC_LDS_MAX - off) / (1024 * tn);
  q.kl = room < 0 ? 0 : (room < ks ? room & ~1 : ks);
  if (a.skip_stages & 64) q.kl = 0;  // timing experiments: every B fragment streamed from L2
  q.lds = off + q.kl * tn * 1024;
  if (q.lds > RC_LDS_MAX) return ENCDIFF_ERR_UNSUPPORTED;
  return ENCDIFF_OK;
}

}  // namespace

#if RC_STAMP
extern "C" int encdiff_debug_rc_stamps(void* dst, int nblocks) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(rc_stamps), (size_t)nblocks * 10 * sizeof(unsigned long long)) == hipSuccess
             ? 0 : -1;
}
extern "C" int encdiff_debug_rc_wstamps(void* dst, int nblocks) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(rc_wstamps), (size_t)nblocks * 64 * sizeof(unsigned long long)) ==
                 hipSuccess ? 0 : -1;
}
#endif

extern "C" int encdiff_resconv_query(const EncdiffResConvArgs* a, int* lds_bytes, int* grid) {
  if (!a) return ENCDIFF_ERR_ARG;
  RcPlan q;
  int tn = 1;
  const int rc = rc_plan(*a, q, tn);
  if (rc != ENCDIFF_OK) return rc;
  if (lds_bytes) *lds_bytes = q.lds;
  if (grid) *grid = (a->cout / (16 * tn)) * q.ngroup * q.nchunk;
  return ENCDIFF_OK;
}

extern "C" int encdiff_resconv_fwd(const EncdiffResConvArgs* a, void* stream) {
  if (!a) return ENCDIFF_ERR_ARG;
  RcPlan q;
  int tn = 1;
  const int rc = rc_plan(*a, q, tn);
  if (rc != ENCDIFF_OK) return rc;
  const int grid = (a->cout / (16 * tn)) * q.ngroup * q.nchunk;
  if (tn == 1) {
    static const hipError_t attr = hipFuncSetAttribute((const void*)resconv_kernel<1>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, RC_LDS_MAX);
    (void)attr;
    hipLaunchKernelGGL(resconv_kernel<1>, dim3(grid), dim3(RC_THREADS), q.lds, (hipStream_t)stream, *a, q);
  } else {
    static const hipError_t attr = hipFuncSetAttribute((const void*)resconv_kernel<2>,
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, RC_LDS_MAX);
    (void)attr;
    hipLaunchKernelGGL(resconv_kernel<2>, dim3(grid), dim3(RC_THREADS), q.lds, (hipStream_t)stream, *a, q);
  }
  ED_CHECK_LAUNCH();
  return ENCDIFF_OK;
}
