// gemm.hip -- one MFMA GEMM engine for every conv / linear of the EncDiff UNet.
//
// C[M][N] = alpha * A[M][K] * B[K][N] (+bias)(+resid), bf16 operands, fp32 accumulate,
// v_mfma_f32_16x16x32_bf16 on gfx950.  256 threads = 4 waves in a 2x2 layout, each
// wave owns a (BM/2)x(BN/2) sub-tile.  K is staged 64 at a time through
// double-buffered LDS with register staging (global_load_dwordx4 -> ds_write_b128).
//
// Operands are loaded in their natural global layout ("k-inner": rows of K,
// read as MFMA fragments with ds_read_b128; "k-outer": rows of M/N, read with the
// gfx950 transpose read ds_read_b64_tr_b16), so the same engine runs
//   forward   conv3x3  : A = implicit im2col(x) [pixels][9*Cin], B = W [Cout][9*Cin]
//   dgrad     conv3x3  : A = im2col(dY),   B = W read through a flipped-tap map
//   wgrad     conv3x3  : A = dY^T (k-outer), B = im2col(x) (k-outer), split-K, atomics
//   linear fwd / dgrad / wgrad likewise with dense operands.
// Replaces: openaimodel_enc.py:204,230,237-241,508-512,521,687; attention.py:159-167,
// 43,58,233-259 (every Conv2d / Linear forward and their autograd backward).
#include "common.h"

#include <algorithm>
#include <cstring>
#include <vector>

namespace {

constexpr int BK = 64;

enum { A_ROWK = ENCDIFF_OPA_ROWK, A_IM2COL = ENCDIFF_OPA_IM2COL, A_ROWM = ENCDIFF_OPA_ROWM };
enum { B_ROWK = ENCDIFF_OPB_ROWK, B_ROWN = ENCDIFF_OPB_ROWN, B_CONVD = ENCDIFF_OPB_CONV_DGRAD,
       B_IM2COL = ENCDIFF_OPB_IM2COL };

// internal A modes: implicit im2col read from a per-workgroup halo image in LDS (tiles >= 16);
// implicit im2col with GroupNorm(+FiLM)(+SiLU) applied to each staged A tile (EncdiffGemmArgs.agn_*)
enum { A_HALO = 16, A_IM2COL_GN = 17, A_ROWK_LN = 18 };

template <int AM> struct AKInner { static constexpr bool v = AM != A_ROWM; };
template <int BMd> struct BKInner { static constexpr bool v = BMd == B_ROWK; };

// LDS tiles are unpadded rows of 16-byte chunks, filled by LDS-DMA (global_load_lds_dwordx4:
// one wave instruction writes 1 KiB lane-linearly).  Bank conflicts of the fragment reads are
// removed by an XOR swizzle applied on the SOURCE side: the chunk stored at LDS slot s of
// row r is the global chunk s ^ (r & 7), and reads apply the same involution.
template <int ROWS, bool KINNER, int KB = BK>
struct TileShape {
  // k-inner: [ROWS][KB]; k-outer: [KB][ROWS]
  static constexpr int LD = KINNER ? KB : ROWS;            // elements per LDS row
  static constexpr int SLOTS = LD / 8;                      // 16-byte chunks per row
  static constexpr int ELEMS = ROWS * KB;
  static constexpr int CHUNKS = ROWS * KB / 8;  // 16-byte chunks per tile
  static constexpr int PER_THREAD = CHUNKS / 256;
  // swizzle mask: 16 rows of a 256-byte k-inner row (KB = 128) spread over all 64 banks;
  // a 4-slot k-outer row (32 columns) swizzles within its 4 slots
  static constexpr int SWM = (KINNER && KB >= 128) ? 15 : (SLOTS < 8 ? SLOTS - 1 : 7);
  // Bank swizzle (an involution on a row's slots): k-inner rows are read by ds_read_b128 along
  // rows (slot ^ row); k-outer rows by ds_read_b64_tr_b16, whose 32-lane groups read rows
  // {r..r+3, r+8..r+11} two slots each -- the XOR keeps each slot pair aligned and gives those
  // 8 rows distinct bank positions (slot ^ (row & 7) put rows r and r+8 on the same banks: ~half
  // the weight-gradient tiles' LDS cycles were conflicts)
  static ED_DEV int sw(int row, int slot) {
    if constexpr (KINNER || LD < 64) return slot ^ (row & SWM);
    else if constexpr (LD == 64) return slot ^ ((((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2));
    else return slot ^ (((row & 3) << 1) | (((row >> 3) & 1) << 3));
  }
};
ED_DEV int swz(int row, int slot, int mask = 7) { return slot ^ (row & mask); }

// 16 zero bytes in global memory: the source of masked (padding / out-of-range) chunks,
// so LDS-DMA lanes never need a branch.
__device__ __attribute__((aligned(16))) const uint4 g_zero16 = {0u, 0u, 0u, 0u};

// ---------------------------------------------------------------------------
// Exact division by a launch constant without a divider: n / d == (n * mul) >> 40 for
// n * d < 2^40 (pixels < 2^24, divisors < 2^16 here); mul = 2^40 / d + 1 from the host.
struct FDiv {
  unsigned long long mul;
  uint32_t d, pad_;
};
ED_DEV uint32_t fdiv(uint32_t n, const FDiv& f) { return (uint32_t)(((unsigned long long)n * f.mul) >> 40); }

// Halo tiles (A_HALO): a workgroup's BM output pixels are R whole rows of one image (or NI
// whole images); every conv-input pixel their taps reach -- an (hr x hc) window per image, all
// cin channels -- is staged into LDS ONCE by LDS-DMA, so the K loop streams only weights and the
// im2col operand is read from L2 once instead of once per tap.  Conv-input coordinate of halo
// pixel (hy, hx): (s*y0 + off + hy, off + hx), bounds (lh, lw); source pixel = coordinate >> ush
// (nearest-up) of an (hs x ws) image.  16-byte chunk c of halo pixel p sits at LDS slot
// c ^ ((p >> xsh) & xmsk): the 16 pixels an MFMA fragment read touches land on distinct banks.
struct HaloGeom {
  int hr, hc, ni;      // halo rows / cols per image, images per tile
  int s, off, kt;      // conv-input stride, window origin offset, taps per dimension
  int lh, lw, ush, hs, ws;
  int ch, xsh, xmsk;   // 16-B chunks per pixel (cin / 8), bank swizzle
  int npix, chunks;    // halo pixels, chunks rounded up to 256 (one per thread per DMA round)
  FDiv fch, fimg, fhc; // / ch, / (hr * hc), / hc
};

// In-kernel split-K combine (EncdiffGemmArgs.split_counters): the user's output of a slab GEMM
struct SplitFold {
  int* cnt;              // per-tile tickets (NULL: a finalize pass combines the slabs)
  void* c;
  long ldc;
  int mode;              // ENCDIFF_OUT_BF16 / F32 / F32_ACCUM
  float alpha;
  const float* bias;
  const bf16_t* resid;
  long ld_resid;
};

struct GemmAux {
  FDiv cin;   // A/B im2col: k (or n) -> (tap, channel)
  FDiv cout;  // B_CONVD: k -> (tap, co)
  FDiv hw;    // pixel -> (image, in-image index)
  FDiv w;     // in-image index -> (y, x)
  HaloGeom halo;
  SplitFold fold;
  int xcd;    // XCD-aware tile order (gemm_kernel / gemm2_kernel): see xcd_remap
};

// Implicit im2col, branch-free.  The launch's resample mode is folded into uniform
// constants once per thread; per chunk the source pixel of output pixel (b, y, x) and
// 3x3 tap (ty, tx) is  ys = sy*y + ty + oy  (limits lh x lw), then >> sh (nearest-up
// source), row = (b*hs + ys)*ws + xs.  Padding gives ok = false and row 0: the load is
// still issued (and masked when written to LDS), so no branch or early wait is needed.
//   K4S2   (Encoder4 Conv2d(k4, s2, p1), openaimodel_enc.py:1002-1009): 4x4 taps at
//          (2y + ty - 1, 2x + tx - 1) of the (2h, 2w) source;
//   K4S2_T (its input gradient): 4x4 taps t' = 15 - t at (y + ty' - 2, x + tx' - 2) of the
//          full-resolution grid, valid only at even coordinates, source pixel = coordinate / 2;
//   K4S2_TP (the same gradient by output parity): the M rows are ordered [parity q][b][y'][x']
//          over the half-resolution grid, and an output row (b, 2y'+py, 2x'+px), q = 2py+px,
//          receives only the 2x2 taps ty' = py + 2jy, tx' = px + 2jx: source (y'+py+jy-1,
//          x'+px+jx-1) of dY, weight tap 15 - (4ty' + tx').  K = 4*cout instead of 16*cout
//          (K4S2_T multiplies 3 zero taps of every 4).  A tile never straddles parities
//          (batch*h*w/4 % 128 == 0), so oy, ox and the weight-tap base are per workgroup.
struct Im2colMode {
  int sy, oy, ox, lh, lw, sh, hs, ws, par, k4, tb;
  ED_DEV Im2colMode(const EncdiffConvGeom& g) {
    const bool s2 = g.resample == ENCDIFF_RESAMPLE_STRIDE2;  // VQ Downsample: pad (0,1,0,1), k3 s2 p0
    const bool up = g.resample == ENCDIFF_RESAMPLE_UP2;      // nearest x2 (openaimodel_enc.py:116)
    const bool f4 = g.resample == ENCDIFF_RESAMPLE_K4S2;
    const bool t4 = g.resample == ENCDIFF_RESAMPLE_K4S2_T;
    const bool tp = g.resample == ENCDIFF_RESAMPLE_K4S2_TP;
    sy = (s2 || f4) ? 2 : 1;
    oy = s2 ? 0 : (t4 ? -2 : -1);
    ox = oy;
    lh = (s2 || f4) ? 2 * g.h : (tp ? g.h >> 1 : g.h);
    lw = (s2 || f4) ? 2 * g.w : (tp ? g.w >> 1 : g.w);
    sh = (up || t4) ? 1 : 0;
    hs = lh >> sh;
    ws = lw >> sh;
    par = t4 ? 1 : 0;
    k4 = tp ? 2 : ((f4 || t4) ? 1 : 0);
    tb = 15;
  }
  // K4S2_TP: the workgroup's parity class q = 2py + px
  ED_DEV void set_parity(int q) {
    oy = (q >> 1) - 1;
    ox = (q & 1) - 1;
    tb = 15 - 4 * (q >> 1) - (q & 1);
  }
  // weight tap of im2col tap `tap` for OPB_CONV_DGRAD (flipped kernel)
  ED_DEV uint32_t wtap(uint32_t tap) const {
    return k4 == 2 ? (uint32_t)tb - 8u * (tap >> 1) - 2u * (tap & 1u) : (k4 ? 15u : 8u) - tap;
  }
};

// tap index -> (ty, tx): 3x3 (tap / 3 via a multiply), 4x4 or 2x2 taps
ED_DEV void tap_yx(const Im2colMode& md, uint32_t tap, int& ty, int& tx) {
  ty = md.k4 ? (int)(tap >> (3 - md.k4)) : (int)((tap * 11u) >> 5);
  tx = (int)tap - (md.k4 ? (1 << (3 - md.k4)) : 3) * ty;
}

ED_DEV uint32_t im2col_row(const Im2colMode& md, uint32_t b, int y, int x, int ty, int tx, bool& ok) {
  const int ys = md.sy * y + ty + md.oy, xs = md.sy * x + tx + md.ox;
  ok = (unsigned)ys < (unsigned)md.lh && (unsigned)xs < (unsigned)md.lw && ((ys | xs) & md.par) == 0;
  const uint32_t row = (b * (uint32_t)md.hs + (uint32_t)(ys >> md.sh)) * (uint32_t)md.ws + (uint32_t)(xs >> md.sh);
  return ok ? row : 0u;
}

template <int BM, int BN, int AM, int BMD, int NS = 2, int KB = BK>
struct Gemm {
  static constexpr bool AKI = AKInner<AM>::v;
  static constexpr bool BKI = BKInner<BMD>::v;
  static constexpr int KT = KB;  // k per LDS stage
  using TA = TileShape<BM, AKI, KB>;
  using TB = TileShape<BN, BKI, KB>;
  static constexpr int TM = BM / 32;  // 16x16 MFMA tiles per wave along M
  static constexpr int TN = BN / 32;
  static constexpr bool HALO = AM == A_HALO;
  static constexpr bool AGN = AM == A_IM2COL_GN;  // GroupNorm applied to the staged A tiles
  static constexpr bool LNA = AM == A_ROWK_LN;    // LayerNorm applied to the staged A tiles (ROWK)
  static constexpr bool IM2 = AM == A_IM2COL || AGN;
  static constexpr int ASTAGE = HALO ? 0 : TA::ELEMS;  // halo mode: the ring holds B only
  static constexpr int STAGE = ASTAGE + TB::ELEMS;     // elements per LDS stage
  // LDS ring depth.  Measured on the step's GEMMs: 3-4 stages for every GEMM (one or two
  // workgroups per CU) lost 7% overall against 2 stages with up to five resident workgroups
  // per CU hiding the load latency instead; the deeper rings are tile choices of their own
  // (tiles 5, 6) that the measured table picks per problem.
  static constexpr int NSTAGE = NS;
  static constexpr int LPS = (HALO ? 0 : TA::PER_THREAD) + TB::PER_THREAD;  // LDS-DMA loads per thread per stage
  // the staging ring, reused by the fp32 epilogue tile [BM][BN + 4]
  static constexpr int LDS_BYTES =
      (NSTAGE * STAGE * 2 > BM * (BN + 4) * 4) ? NSTAGE * STAGE * 2 : BM * (BN + 4) * 4;
};

// ds_read_b64_tr_b16 as inline asm.  Through the builtin, hipcc cannot tell the transposed read
// from the LDS-DMA writes still in flight to ANOTHER ring slot and drains them (s_waitcnt
// vmcnt(0)) before every k-outer fragment read: the next stage's loads then never overlap the
// current tile's MFMAs in any backward GEMM.  The asm read is waited for explicitly (compute()).
ED_DEV v4s ds_read_tr16(const bf16_t* p) {
  typedef __attribute__((address_space(3))) const char lds_char;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_char*)p;
  v4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a));
  return r;
}

// ds_read_b128 as inline asm, for tiles whose fragment waits are counted by hand (compute()):
// a compiler-issued read would be waited for by the compiler, which does not count the asm reads.
ED_DEV v8bf ds_read_b128(const bf16_t* p) {
  typedef __attribute__((address_space(3))) const char lds_char;
  const uint32_t a = (uint32_t)(uintptr_t)(lds_char*)p;
  v4u32 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a));
  return __builtin_bit_cast(v8bf, r);
}

// Fragment reads software-pipelined across k-substeps (compute()): measured in the step with both
// builds on one box (round 4, tools/bench_ab.sh): 9.516-9.524 ms/step pipelined vs 9.503-9.522
// without -- no gain (five resident workgroups per CU already hide the LDS latency) for 4-12 more
// VGPRs, so it is off; -DED_FRAG_PIPE=1 builds it.
#ifndef ED_FRAG_PIPE
#define ED_FRAG_PIPE 0
#endif

// Wait until at most N of this thread's vector-memory loads are outstanding (LDS-DMA stages
// still in flight behind the one about to be read).
template <int N>
ED_DEV void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int LPS, int MAXA = 2>
ED_DEV void vm_wait_stages(int ahead) {
  // ahead = stages still allowed in flight behind the one about to be read (<= ring depth - 2)
  if (MAXA >= 6 && ahead >= 6) vm_wait<6 * LPS>();
  else if (MAXA >= 5 && ahead == 5) vm_wait<5 * LPS>();
  else if (MAXA >= 4 && ahead == 4) vm_wait<4 * LPS>();
  else if (MAXA >= 3 && ahead == 3) vm_wait<3 * LPS>();
  else if (ahead >= 2) vm_wait<2 * LPS>();
  else if (ahead == 1) vm_wait<LPS>();
  else vm_wait<0>();
}

// One output tile (bx, by) of split bz.  Shared by the single-GEMM kernel and the paired
// kernel that runs two independent GEMMs (a layer's input- and weight-gradient) in one grid.
template <int BM, int BN, int AM, int BMD, int NS = 2, int KB = BK>
__device__ __forceinline__ void gemm_tile(const EncdiffGemmArgs& p, const GemmAux& aux, const int bx, const int by,
                                          const int bz, bf16_t* smem) {
  using G = Gemm<BM, BN, AM, BMD, NS, KB>;
  constexpr int BK = G::KT;  // shadows the default stage depth
  using TA = typename G::TA;
  using TB = typename G::TB;
  constexpr bool AKI = G::AKI, BKI = G::BKI;
  constexpr int TM = G::TM, TN = G::TN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = (wave >> 1) * (BM / 2);
  const int wc = (wave & 1) * (BN / 2);
  const int m0 = bx * BM;
  const int n0 = by * BN;

  // split-K range
  const int ktiles_total = (p.K + BK - 1) / BK;
  const int kt_per = (ktiles_total + p.split_k - 1) / p.split_k;
  const int kt_begin = bz * kt_per;
  const int kt_end = min(ktiles_total, kt_begin + kt_per);
  int nkt = kt_end - kt_begin;
  // halo tiles with split-K: split bz owns the source channels [hcb, hcb + 8 h.ch) of every tap
  // (the window holds that slice only); its k-tiles run tap by tap over the slice's 64-channel
  // groups, k-tile (tap, g) = tap * cin / 64 + bz * ncc + g
  uint32_t hcb = 0;
  int kt_ncc = 0, kt_c64 = 0;
  if constexpr (G::HALO) {
    if (p.split_k > 1) {
      kt_ncc = aux.halo.ch >> 3;
      kt_c64 = p.conv.cin >> 6;
      hcb = (uint32_t)(bz * aux.halo.ch * 8);
      nkt = aux.halo.kt * aux.halo.kt * kt_ncc;
    }
  }
  auto ktile = [&](int it) -> int {
    if constexpr (G::HALO) {
      if (kt_ncc) {
        const int tap = it / kt_ncc;
        return tap * kt_c64 + bz * kt_ncc + (it - tap * kt_ncc);
      }
    }
    return kt_begin + it;
  };

  const bf16_t* __restrict__ A = (const bf16_t*)p.a;
  const bf16_t* __restrict__ B = (const bf16_t*)p.b;

  Im2colMode md(p.conv);
  // K4S2_TP: rows [parity][b][y'][x'], one parity per tile (host: batch*h*w/4 % 128 == 0)
  const int tp_q = md.k4 == 2 ? m0 / (p.M >> 2) : 0;
  const uint32_t mbase = md.k4 == 2 ? (uint32_t)(tp_q * (p.M >> 2)) : 0u;
  if (md.k4 == 2) md.set_parity(tp_q);

  // LDS-DMA staging: every chunk's global address is computed branch-free (masked chunks
  // read g_zero16) and copied straight into the lane-linear LDS image; tile t+1 is in
  // flight while tile t is multiplied (depth-1 prefetch, no staging VGPRs).
  typedef __attribute__((address_space(3))) void lds_void;
  typedef __attribute__((address_space(1))) const void gbl_void;
  // GEGLU proj (OUT_BF16_GEGLU): tile column c < BN/2 is value column by*BN/2 + c of f, the
  // rest gate column N/2 + by*BN/2 + c - BN/2, so one tile holds both halves of its outputs
  const bool gfwd = p.c_mode == ENCDIFF_OUT_BF16_GEGLU;
  auto gcol = [&](int c) -> int {
    return c < BN / 2 ? by * (BN / 2) + c : (p.N >> 1) + by * (BN / 2) + c - BN / 2;
  };
  // halo mode: the window sits at the LDS base, the B ring behind it
  bf16_t* ring = smem;
  if constexpr (G::HALO) ring = smem + aux.halo.chunks * 8;
  auto stage_halo = [&]() {
    const HaloGeom& h = aux.halo;
    const uint32_t b0 = fdiv((uint32_t)m0, aux.hw);
    const uint32_t y0 = fdiv((uint32_t)m0 - b0 * aux.hw.d, aux.w);  // 0 when the tile holds whole images
    const int cy0 = h.s * (int)y0 + h.off;
    for (int c = tid; c < h.chunks; c += 256) {
      const uint32_t px = fdiv((uint32_t)c, h.fch);
      const int gch = (c - (int)(px * (uint32_t)h.ch)) ^ ((int)(px >> h.xsh) & h.xmsk);
      const uint32_t j = fdiv(px, h.fimg);
      const uint32_t r = px - j * h.fimg.d;
      const uint32_t hy = fdiv(r, h.fhc);
      const int cy = cy0 + (int)hy, cx = h.off + (int)(r - hy * (uint32_t)h.hc);
      const bool ok = (int)px < h.npix && (unsigned)cy < (unsigned)h.lh && (unsigned)cx < (unsigned)h.lw;
      const uint32_t row = ((b0 + j) * (uint32_t)h.hs + (uint32_t)(cy >> h.ush)) * (uint32_t)h.ws + (uint32_t)(cx >> h.ush);
      const void* src = ok ? (const void*)(A + (size_t)row * p.conv.ld_src + hcb + gch * 8) : (const void*)&g_zero16;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(smem + (c & ~63) * 8), 16, 0, 0);
    }
  };
  // Staging addresses.  Buffer-resource LDS-DMA with 32-bit byte offsets (host: every operand
  // spans < 2^31 bytes); a masked chunk (padding tap, tile tail) gets an out-of-range offset and
  // the DMA writes zeros.  What does not depend on the k-tile is computed once per thread here,
  // so a chunk costs a few adds and compares per k-tile: the earlier form (64-bit addresses, a
  // zero-page pointer per masked chunk, the pixel / tap decomposition redone per chunk) issued
  // 20-30 VALU per 16-byte chunk and left the MFMA pipe idle behind the address arithmetic.
  constexpr uint32_t OOB = 0x80000000u;
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, 0x7FFFFFF0, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, 0x7FFFFFF0, 0x00020000);
  constexpr int APT = G::HALO ? 0 : TA::PER_THREAD, BPT = TB::PER_THREAD;
  const uint32_t ldsrc2 = (uint32_t)p.conv.ld_src * 2u;
  // a k-tile of an im2col / flipped-weight operand lies inside one tap: tap and channel base are
  // uniform per k-tile
  const bool a_tapk = G::IM2 && (p.conv.cin % BK) == 0;
  const bool b_tapk = BMD == B_CONVD && (p.conv_cout % BK) == 0;
  // weight-gradient im2col operand (k = output pixel): with w | BK and hw | BK or BK | hw, pixel
  // k0 + r splits into a uniform part of k0 and a per-lane part of r (no per-k-tile division)
  bool b_pix = false;
  if constexpr (BMD == B_IM2COL) b_pix = (BK % aux.w.d) == 0 && ((aux.hw.d % BK) == 0 || (BK % aux.hw.d) == 0);
  uint32_t a_off[APT > 0 ? APT : 1];  // invariant byte offset (OOB: masked row)
  int a_k[APT > 0 ? APT : 1], a_y[APT > 0 ? APT : 1], a_x[APT > 0 ? APT : 1];
  int a_bl[APT > 0 ? APT : 1];  // AGN: the chunk row's image, relative to the tile's first image
  uint32_t agn_b0 = 0;          // AGN: the tile's first image
  uint32_t b_off[BPT], b_n2[BPT];
  int b_k[BPT], b_ys[BPT];
  uint32_t b_base[BPT], b_xsh[BPT];
#pragma unroll
  for (int i = 0; i < APT; ++i) {
    const int c = tid + 256 * i;
    const int row = c / TA::SLOTS, slot = c % TA::SLOTS;
    const int gs = TA::sw(row, slot);
    if constexpr (AM == A_ROWK || AM == A_ROWK_LN) {
      const int m = m0 + row;
      a_y[i] = row;  // LNA: the chunk's tile row (its LayerNorm statistics)
      a_k[i] = gs * 8;
      a_off[i] = m < p.M ? ((uint32_t)m * (uint32_t)p.lda + (uint32_t)(gs * 8)) * 2u : OOB;
    } else if constexpr (AM == A_ROWM) {
      const int m = m0 + gs * 8;
      a_k[i] = row;
      a_off[i] = m < p.M ? ((uint32_t)row * (uint32_t)p.lda + (uint32_t)m) * 2u : OOB;
    } else if constexpr (G::IM2) {  // this row = output pixel (fixed): source window origin
      const uint32_t mm0 = (uint32_t)(m0 + row);
      const bool min = mm0 < (uint32_t)p.M;
      const uint32_t mm = min ? mm0 - mbase : 0u;
      const uint32_t bb = fdiv(mm, aux.hw);
      if constexpr (G::AGN) a_bl[i] = (int)(bb - fdiv((uint32_t)m0, aux.hw));
      const uint32_t r = mm - bb * aux.hw.d;
      const int y = (int)fdiv(r, aux.w), x = (int)(r - (uint32_t)y * aux.w.d);
      a_k[i] = gs * 8;
      a_y[i] = min ? md.sy * y + md.oy : (1 << 28);  // out of range: masked row
      a_x[i] = md.sy * x + md.ox;
      a_off[i] = bb * (uint32_t)md.hs;
    }
  }
#pragma unroll
  for (int i = 0; i < BPT; ++i) {
    const int c = tid + 256 * i;
    const int row = c / TB::SLOTS, slot = c % TB::SLOTS;
    const int gs = TB::sw(row, slot);
    if constexpr (BKI) {  // B_ROWK: Bt[n][k], row = n
      const int n = gfwd ? gcol(row) : n0 + row;
      b_k[i] = gs * 8;
      b_off[i] = n < p.N ? ((uint32_t)n * (uint32_t)p.ldb + (uint32_t)(gs * 8)) * 2u : OOB;
    } else {  // k-outer: row = k, chunk = 8 columns of n
      const int n = n0 + gs * 8;
      b_k[i] = row;
      if constexpr (BMD == B_ROWN || BMD == B_CONVD) {
        b_off[i] = n < p.N ? ((uint32_t)row * (uint32_t)p.ldb + (uint32_t)n) * 2u : OOB;
        b_n2[i] = n < p.N ? (uint32_t)n * 2u : OOB;
      } else {  // B_IM2COL: column n = (tap, ci), invariant; row = pixel offset in the k-tile
        const uint32_t nn = n < p.N ? (uint32_t)n : 0u;
        const uint32_t tap = fdiv(nn, aux.cin);
        const uint32_t ci = nn - tap * (uint32_t)p.conv.cin;
        int ty, tx;
        tap_yx(md, tap, ty, tx);
        b_n2[i] = n < p.N ? ci * 2u : OOB;
        b_off[i] = (uint32_t)(ty * 16 + tx);  // general path: tap offsets
        if (b_pix) {
          const uint32_t bl = fdiv((uint32_t)row, aux.hw), rl = (uint32_t)row - bl * aux.hw.d;
          const uint32_t yl = fdiv(rl, aux.w), xl = rl - yl * aux.w.d;
          const int xs = md.sy * (int)xl + tx + md.ox;
          const bool xok = (unsigned)xs < (unsigned)md.lw && (xs & md.par) == 0 && n < p.N;
          b_ys[i] = xok ? md.sy * (int)yl + ty + md.oy : (1 << 28);
          b_base[i] = bl * (uint32_t)md.hs;
          b_xsh[i] = (uint32_t)(xs >> md.sh);
        }
      }
    }
  }
  auto stage = [&](bf16_t* s, int kt) {
    const int k0 = kt * BK;
    bf16_t* sa = s;
    bf16_t* sb = s + G::ASTAGE;
    // uniform per-k-tile values
    uint32_t a_ch = 0u, b_cv = 0u, b_pb = 0u;
    int a_ty = 0, a_tx = 0, b_yo = 0;
    if constexpr (G::IM2) {
      if (a_tapk) {
        const uint32_t tap = fdiv((uint32_t)k0, aux.cin);
        a_ch = (uint32_t)k0 - tap * (uint32_t)p.conv.cin;
        tap_yx(md, tap, a_ty, a_tx);
      }
    }
    if constexpr (BMD == B_CONVD) {
      if (b_tapk) {
        const uint32_t tap = fdiv((uint32_t)k0, aux.cout);
        const uint32_t co = (uint32_t)k0 - tap * (uint32_t)p.conv_cout;
        b_cv = (co * (uint32_t)p.ldb + md.wtap(tap) * (uint32_t)p.N) * 2u;
      }
    }
    if constexpr (BMD == B_IM2COL) {
      if (b_pix) {
        const uint32_t bs = fdiv((uint32_t)k0, aux.hw);
        const uint32_t ys = fdiv((uint32_t)k0 - bs * aux.hw.d, aux.w);
        b_yo = md.sy * (int)ys;
        b_pb = bs * (uint32_t)md.hs;
      }
    }
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int c = tid + 256 * i;  // LDS chunk position (lane-linear)
      const int k = k0 + a_k[i];
      uint32_t vo;
      if constexpr (AM == A_ROWK || AM == A_ROWK_LN) {
        vo = k < p.K ? a_off[i] + 2u * (uint32_t)k0 : OOB;
      } else if constexpr (AM == A_ROWM) {
        vo = k < p.K ? a_off[i] + (uint32_t)k0 * (uint32_t)p.lda * 2u : OOB;
      } else {  // IM2COL
        uint32_t ch;
        int ty, tx;
        if (a_tapk) {
          ch = a_ch + (uint32_t)a_k[i];
          ty = a_ty;
          tx = a_tx;
        } else {
          const uint32_t kk = k < p.K ? (uint32_t)k : 0u;
          const uint32_t tap = fdiv(kk, aux.cin);
          ch = kk - tap * (uint32_t)p.conv.cin;
          tap_yx(md, tap, ty, tx);
        }
        const int ys = a_y[i] + ty, xs = a_x[i] + tx;
        const bool ok = k < p.K && (unsigned)ys < (unsigned)md.lh && (unsigned)xs < (unsigned)md.lw &&
                        ((ys | xs) & md.par) == 0;
        const uint32_t prow = (a_off[i] + (uint32_t)(ys >> md.sh)) * (uint32_t)md.ws + (uint32_t)(xs >> md.sh);
        vo = ok ? prow * ldsrc2 + ch * 2u : OOB;
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(sa + (c & ~63) * 8), 16, vo, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < BPT; ++i) {
      const int c = tid + 256 * i;
      const int k = k0 + b_k[i];
      uint32_t vo;
      if constexpr (BKI) {
        vo = k < p.K ? b_off[i] + 2u * (uint32_t)k0 : OOB;
      } else if constexpr (BMD == B_ROWN) {
        vo = k < p.K ? b_off[i] + (uint32_t)k0 * (uint32_t)p.ldb * 2u : OOB;
      } else if constexpr (BMD == B_CONVD) {
        if (b_tapk) {
          vo = k < p.K ? b_off[i] + b_cv : OOB;
        } else {
          const uint32_t kk = k < p.K ? (uint32_t)k : 0u;
          const uint32_t tap = fdiv(kk, aux.cout);
          const uint32_t co = kk - tap * (uint32_t)p.conv_cout;
          vo = k < p.K ? b_n2[i] + (co * (uint32_t)p.ldb + md.wtap(tap) * (uint32_t)p.N) * 2u : OOB;
        }
      } else {  // B_IM2COL
        if (b_pix) {
          const int ys = b_ys[i] + b_yo;
          const bool ok = k < p.K && (unsigned)ys < (unsigned)md.lh && (ys & md.par) == 0;
          const uint32_t prow = (b_pb + b_base[i] + (uint32_t)(ys >> md.sh)) * (uint32_t)md.ws + b_xsh[i];
          vo = ok ? prow * ldsrc2 + b_n2[i] : OOB;
        } else {
          const uint32_t kk = k < p.K ? (uint32_t)k : 0u;
          const uint32_t bb = fdiv(kk, aux.hw);
          const uint32_t r = kk - bb * aux.hw.d;
          const int y = (int)fdiv(r, aux.w), x = (int)(r - (uint32_t)y * aux.w.d);
          const int ty = (int)(b_off[i] >> 4), tx = (int)(b_off[i] & 15u);
          bool inb;
          const uint32_t prow = im2col_row(md, bb, y, x, ty, tx, inb);
          vo = (k < p.K && inb) ? prow * ldsrc2 + b_n2[i] : OOB;
        }
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void*)(sb + (c & ~63) * 8), 16, vo, 0, 0, 0);
    }
  };

  v4f acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  // optional bias-gradient: column sums of the (k-outer) A operand over K
  const bool do_bgrad = (AM == A_ROWM) && p.bias_grad != nullptr && by == 0;
  float bsum = 0.f;

  const int l16 = lane & 15;
  const int g4 = lane >> 4;
  const int tq = l16 >> 2, tp = l16 & 3;  // transpose-read address roles

  auto frag_kinner = [&](const bf16_t* s, int row, int kk, int mask) -> v8bf {
    return *(const v8bf*)(s + row * BK + swz(row, kk * 4 + g4, mask) * 8);
  };
  auto frag_kinner_asm = [&](const bf16_t* s, int row, int kk, int mask) -> v8bf {
    return ds_read_b128(s + row * BK + swz(row, kk * 4 + g4, mask) * 8);
  };
  auto frag_kouter = [&](auto tile, const bf16_t* s, int colbase, int kk) -> v8bf {
    // rows k = kk*32 + g4*8 + tq (+4): 4 bf16 at column colbase + 4*tp, swizzled chunk
    using T = decltype(tile);
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const int r0 = kk * 32 + g4 * 8 + tq, r1 = r0 + 4;
    const int ch = (colbase >> 3) + (tp >> 1), sub = (tp & 1) * 4;
    v4s lo = ds_read_tr16(s + r0 * T::LD + T::sw(r0, ch) * 8 + sub);
    v4s hi = ds_read_tr16(s + r1 * T::LD + T::sw(r1, ch) * 8 + sub);
    v8s r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(v8bf, r);
  };

  // halo mode: window pixel of each of this lane's fragment rows at tap (0, 0)
  uint32_t hpb[TM];
  if constexpr (G::HALO) {
    const HaloGeom& h = aux.halo;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const uint32_t m = (uint32_t)(wr + 16 * i + l16);
      const uint32_t j = fdiv(m, aux.hw), rr = m - j * aux.hw.d;
      const uint32_t ry = fdiv(rr, aux.w), rx = rr - ry * aux.w.d;
      hpb[i] = j * h.fimg.d + (uint32_t)h.s * (ry * (uint32_t)h.hc + rx);
    }
  }
  auto frag_halo = [&](int kt, int kk, int i) -> v8bf {
    const HaloGeom& h = aux.halo;
    uint32_t k = (uint32_t)(kt * BK + kk * 32 + g4 * 8);
    if (k >= (uint32_t)p.K) k = 0;  // tail of the last k-tile: B is zero there, keep A finite
    const uint32_t tap = fdiv(k, aux.cin), ci = k - tap * (uint32_t)p.conv.cin - hcb;
    const uint32_t ty = h.kt == 4 ? tap >> 2 : (tap * 11u) >> 5;
    const uint32_t hp = hpb[i] + ty * (uint32_t)h.hc + (tap - (uint32_t)h.kt * ty);
    const uint32_t slot = (ci >> 3) ^ ((hp >> h.xsh) & (uint32_t)h.xmsk);
    return *(const v8bf*)(smem + (hp * (uint32_t)h.ch + slot) * 8);
  };

  auto compute = [&](const bf16_t* s, int kt) {
    const bf16_t* sa = s;
    const bf16_t* sb = s + G::ASTAGE;
    if (do_bgrad) {
      // BM columns x BK rows; 256 threads -> 256/BM row-groups
      constexpr int RG = 256 / BM;
      const int col = tid % BM, rg = tid / BM;
#pragma unroll 4
      for (int r = rg * (BK / RG); r < (rg + 1) * (BK / RG); ++r)
        bsum += bf2f(sa[r * TA::LD + TA::sw(r, col >> 3) * 8 + (col & 7)]);
    }
    constexpr int KK = BK / 32;
    if constexpr (ED_FRAG_PIPE && (!AKI || !BKI) && !G::HALO && KK > 1) {
      // Tiles with a transposed (k-outer) operand read every fragment by inline asm, so the
      // waits are ours: the fragments of k-substep kk+1 are issued BEFORE the MFMAs of kk, which
      // wait only for kk's reads (counted lgkmcnt: LDS returns in order) -- the LDS latency of
      // the next substep hides behind this one's MFMAs instead of draining to zero each time.
      constexpr int RA = AKI ? 1 : 2, RB = BKI ? 1 : 2;
      constexpr int NR = TM * RA + TN * RB;          // LDS read instructions per substep
      constexpr int NW = NR > 15 ? 15 : NR;           // lgkmcnt is 4 bits: over-wait when larger
      v8bf af[2][TM], bfr[2][TN];
      auto load = [&](int kk, v8bf* a, v8bf* b) {
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          if constexpr (AKI) a[i] = frag_kinner_asm(sa, wr + 16 * i + l16, kk, TA::SWM);
          else a[i] = frag_kouter(TA{}, sa, wr + 16 * i, kk);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          if constexpr (BKI) b[j] = frag_kinner_asm(sb, wc + 16 * j + l16, kk, TB::SWM);
          else b[j] = frag_kouter(TB{}, sb, wc + 16 * j, kk);
        }
      };
      load(0, af[0], bfr[0]);
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int cur = kk & 1;
        if (kk + 1 < KK) {
          load(kk + 1, af[cur ^ 1], bfr[cur ^ 1]);
          asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(NW) : "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[cur][i], bfr[cur][j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      return;
    }
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      v8bf af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        if constexpr (G::HALO) af[i] = frag_halo(kt, kk, i);
        else if constexpr (AKI) af[i] = frag_kinner(sa, wr + 16 * i + l16, kk, TA::SWM);
        else af[i] = frag_kouter(TA{}, sa, wr + 16 * i, kk);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (BKI) bfr[j] = frag_kinner(sb, wc + 16 * j + l16, kk, TB::SWM);
        else bfr[j] = frag_kouter(TB{}, sb, wc + 16 * j, kk);
      }
      if constexpr (!AKI || !BKI) {  // asm transposed reads: wait for them before the MFMAs use them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  // AGN (EncdiffGemmArgs.agn_*): GroupNorm32(+FiLM)(+SiLU) of the im2col source, folded into the
  // staging.  Prologue: the statistics of every image the tile's rows read, from x itself (per
  // channel sum / sum of squares over the image's pixels -- thread = (8-channel vector, pixel
  // lane), lanes added in order -- then per group), turned into per-(image, channel) affine
  // coefficients z = x * mul + add (mul = rstd gamma (1 + scale), add = (beta - mean rstd gamma)
  // (1 + scale) + shift) in LDS behind the ring.  Per k-tile: every thread rewrites its own staged
  // A chunks in place (after its LDS-DMA landed, before the barrier that publishes the tile);
  // zero-padding chunks stay zero.
  float2* agn_coef = (float2*)((char*)smem + G::LDS_BYTES);
  if constexpr (G::AGN) {
    const int cin = p.conv.cin, nv = cin >> 3, cpg = cin >> 5;
    const int shw = md.hs * md.ws;  // source image pixels (UP2: the half-resolution image)
    const uint32_t last = min((uint32_t)(m0 + BM), (uint32_t)p.M) - 1u;
    agn_b0 = fdiv((uint32_t)m0, aux.hw);
    const int nimg = (int)fdiv(last, aux.hw) - (int)agn_b0 + 1;
    const int tv = tid % nv, tp = tid / nv, np = 256 / nv;  // host: cin <= 1024
    // pixel lanes per image: every image of the tile in ONE pass of loads (small levels hold many
    // images per 64-row tile; a loop over images serialised a global round trip per image)
    const int lpi = np / nimg > 0 ? np / nimg : 1, ipass = np / lpi;
    float* red = (float*)smem;        // [2][np][cin] per-lane partials (the ring is not staged yet)
    float* gst = red + 2 * np * cin;  // [nimg][32][2]
    float2* chs = agn_coef;           // [nimg][cin] (sum, sum of squares), then the coefficients
    const long lds = p.conv.ld_src;
    for (int j0 = 0; j0 < nimg; j0 += ipass) {
      const int j = j0 + tp / lpi, li = tp - (tp / lpi) * lpi;
      float sa[8], sq[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) sa[i] = sq[i] = 0.f;
      if (tp < ipass * lpi && j < nimg) {
        const bf16_t* xb = A + (size_t)(agn_b0 + j) * shw * lds + tv * 8;
        for (int px0 = li; px0 < shw; px0 += 8 * lpi) {
          uint4 u[8];
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            const int px = px0 + r * lpi;
            u[r] = px < shw ? *(const uint4*)(xb + (size_t)px * lds) : make_uint4(0u, 0u, 0u, 0u);
          }
#pragma unroll
          for (int r = 0; r < 8; ++r) {
            float v[8];
            unpack8(u[r], v);
#pragma unroll
            for (int i = 0; i < 8; ++i) { sa[i] += v[i]; sq[i] += v[i] * v[i]; }
          }
        }
      }
      if (tp < np) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          red[tp * cin + tv * 8 + i] = sa[i];
          red[(np + tp) * cin + tv * 8 + i] = sq[i];
        }
      }
      __syncthreads();
      for (int e = tid; e < ipass * cin; e += 256) {  // (image, channel): its lanes added in order
        const int jj = e / cin, c = e - jj * cin;
        if (j0 + jj < nimg) {
          float a = 0.f, q = 0.f;
          for (int r = jj * lpi; r < (jj + 1) * lpi; ++r) { a += red[r * cin + c]; q += red[(np + r) * cin + c]; }
          chs[(j0 + jj) * cin + c] = make_float2(a, q);
        }
      }
      __syncthreads();
    }
    for (int e = tid; e < nimg * 32; e += 256) {  // (image, group) statistics
      const int j = e >> 5, g = e & 31;
      float a = 0.f, q = 0.f;
      for (int c = g * cpg; c < (g + 1) * cpg; ++c) { const float2 v = chs[j * cin + c]; a += v.x; q += v.y; }
      const float inv = 1.f / ((float)shw * (float)cpg);
      const float mean = a * inv, var = fmaxf(q * inv - mean * mean, 0.f);
      gst[2 * e] = mean;
      gst[2 * e + 1] = rsqrtf(var + p.agn_eps);
    }
    __syncthreads();
    for (int e = tid; e < nimg * cin; e += 256) {  // coefficients, in place of the channel sums
      const int j = e / cin, c = e - j * cin, g = c / cpg, b = (int)agn_b0 + j;
      float mul = gst[2 * (j * 32 + g) + 1] * p.agn_gamma[c];
      float add = p.agn_beta[c] - gst[2 * (j * 32 + g)] * mul;
      if (p.agn_film) {
        const float sc = 1.f + p.agn_film[(long)b * p.ld_agn_film + c];
        mul *= sc;
        add = add * sc + p.agn_film[(long)b * p.ld_agn_film + cin + c];
      }
      agn_coef[e] = make_float2(mul, add);
    }
    __syncthreads();  // the ring is staged next
  }
  auto agn_transform = [&](bf16_t* sa, int kt) {
    const int k0 = kt * BK;
    uint32_t ch0 = 0u;
    int ty0 = 0, tx0 = 0;
    if (a_tapk) {
      const uint32_t tap = fdiv((uint32_t)k0, aux.cin);
      ch0 = (uint32_t)k0 - tap * (uint32_t)p.conv.cin;
      tap_yx(md, tap, ty0, tx0);
    }
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int k = k0 + a_k[i];
      if (k >= p.K) continue;
      uint32_t ch;
      int ty, tx;
      if (a_tapk) {
        ch = ch0 + (uint32_t)a_k[i];
        ty = ty0;
        tx = tx0;
      } else {
        const uint32_t tap = fdiv((uint32_t)k, aux.cin);
        ch = (uint32_t)k - tap * (uint32_t)p.conv.cin;
        tap_yx(md, tap, ty, tx);
      }
      const int ys = a_y[i] + ty, xs = a_x[i] + tx;
      if ((unsigned)ys >= (unsigned)md.lh || (unsigned)xs >= (unsigned)md.lw) continue;  // zero padding / masked row
      bf16_t* q = sa + (tid + 256 * i) * 8;  // this thread's LDS-DMA chunk (lane-linear)
      float v[8];
      unpack8(*(const uint4*)q, v);
      const float2* cf = agn_coef + a_bl[i] * p.conv.cin + ch;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 m = cf[e];
        const float z = v[e] * m.x + m.y;
        v[e] = p.agn_silu ? silu_f(z) : z;
      }
      *(uint4*)q = pack8(v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the rewrites land before the barrier publishes them
  };

  // LNA (EncdiffGemmArgs.lna_*): LayerNorm of the A rows over K, folded into the staging.
  // Prologue: 4 lanes per tile row sum the row (fp32 sum / sum of squares, xor-shuffles over the
  // 4 lanes), mean / rstd per row and gamma / beta per channel into LDS behind the ring.  Per
  // k-tile every thread rewrites its own staged chunks in place (as AGN), masked rows / the K
  // tail left as staged (zeros).
  float2* lna_row = (float2*)((char*)smem + G::LDS_BYTES);  // [BM] (mean, rstd)
  float2* lna_gb = lna_row + BM;                             // [K] (gamma, beta)
  if constexpr (G::LNA) {
    static_assert(BM * 4 == 256, "LNA: 4 lanes per tile row");
    const int r = tid >> 2, q = tid & 3;
    const int m = m0 + r;
    float sa = 0.f, sq = 0.f;
    if (m < p.M) {
      const bf16_t* xr = A + (size_t)m * p.lda;
      for (int k = 8 * q; k < p.K; k += 32) {
        float v[8];
        unpack8(*(const uint4*)(xr + k), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) { sa += v[e]; sq += v[e] * v[e]; }
      }
    }
    sa += __shfl_xor(sa, 1, 64); sq += __shfl_xor(sq, 1, 64);
    sa += __shfl_xor(sa, 2, 64); sq += __shfl_xor(sq, 2, 64);
    if (q == 0) {
      const float inv = 1.f / (float)p.K;
      const float mean = sa * inv, var = fmaxf(sq * inv - mean * mean, 0.f);
      lna_row[r] = make_float2(mean, rsqrtf(var + p.lna_eps));
    }
    for (int k = tid; k < p.K; k += 256) lna_gb[k] = make_float2(p.lna_gamma[k], p.lna_beta[k]);
    __syncthreads();  // the ring is staged next
  }
  auto lna_transform = [&](bf16_t* sa, int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < APT; ++i) {
      const int k = k0 + a_k[i];
      if (k >= p.K || m0 + a_y[i] >= p.M) continue;
      bf16_t* q = sa + (tid + 256 * i) * 8;  // this thread's LDS-DMA chunk (lane-linear)
      float v[8];
      unpack8(*(const uint4*)q, v);
      const float2 st = lna_row[a_y[i]];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float2 gb = lna_gb[k + e];
        v[e] = (v[e] - st.x) * st.y * gb.x + gb.y;
      }
      *(uint4*)q = pack8(v);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  };

  // NSTAGE-deep LDS ring: tiles it+1 .. it+NSTAGE-2 stay in flight while tile it is
  // multiplied, so the K loop is bound by MFMA / bandwidth rather than by one load latency
  // per k-tile.  Per iteration: wait for tile it (vmcnt = loads issued after it), one
  // barrier (tile it visible to all waves; every wave is done with tile it-1, whose slot is
  // refilled next), issue tile it+NSTAGE-1, multiply tile it.
  constexpr int D = G::NSTAGE;
  static_assert(D - 2 <= 6 && (D - 2) * G::LPS <= 63, "vm_wait_stages covers up to six stages ahead");
  if (nkt > 0) {
    // halo mode: the window's DMAs are issued first, so the wait for ring tile 0 covers them
    if constexpr (G::HALO) stage_halo();
#pragma unroll
    for (int st = 0; st < D - 1; ++st)
      if (st < nkt) stage(ring + st * G::STAGE, ktile(st));
    int rd = 0, wr = D - 1;  // ring slots of the tile read now / the tile issued next
    for (int it = 0; it < nkt; ++it) {
      vm_wait_stages<G::LPS, D - 2>(min(D - 2, nkt - 1 - it));
      if constexpr (G::AGN) agn_transform(ring + rd * G::STAGE, kt_begin + it);
      if constexpr (G::LNA) lna_transform(ring + rd * G::STAGE, kt_begin + it);
      asm volatile("s_barrier" ::: "memory");  // (asm: the compiler may not move LDS-DMA issue across it)
      if (it + D - 1 < nkt) stage(ring + wr * G::STAGE, ktile(it + D - 1));
      compute(ring + rd * G::STAGE, ktile(it));
      // this wave's fragment reads of slot rd retire before it reaches the next barrier
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      rd = rd + 1 == D ? 0 : rd + 1;
      wr = wr + 1 == D ? 0 : wr + 1;
    }
    __syncthreads();  // every wave is done with the ring before the epilogue reuses it
  }

  if (do_bgrad) {
    // column sums of the k-outer A: rows 0..RG-1 of each column partial -> combine in LDS
    // order, then ONE writer per column: a split-K slab (summed in order by the finalize),
    // a plain += (single K range), or an atomic for the atomic output modes.
    constexpr int RG = 256 / BM;
    float* red = (float*)smem;  // staging buffers are free after the last barrier
    const int col = tid % BM, rg = tid / BM;
    red[rg * BM + col] = bsum;
    __syncthreads();
    if (rg == 0 && m0 + col < p.M) {
      float t = 0.f;
#pragma unroll
      for (int r = 0; r < RG; ++r) t += red[r * BM + col];
      const bool slab = p.split_k > 1 && p.c == (void*)p.workspace;
      if (slab)
        p.workspace[(long)p.split_k * p.M * p.N + (long)bz * p.M + m0 + col] = t;
      else if (p.c_mode == ENCDIFF_OUT_F32_ATOMIC || p.c_mode == ENCDIFF_OUT_F32_ATOMIC_CONVW || p.split_k > 1)
        atomicAdd(p.bias_grad + m0 + col, t);
      else
        p.bias_grad[m0 + col] += t;
    }
    __syncthreads();
  }

  // ---- epilogue -------------------------------------------------------------
  // Stage the fp32 tile through LDS (the staging buffers are free after the last barrier),
  // then write whole 16-byte row segments (bf16/fp32 outputs) or lane-contiguous fp32 atomics.
  const bool add_bias = p.bias != nullptr && bz == 0;
  const bf16_t* R = (const bf16_t*)p.resid;
  if (p.c_mode == ENCDIFF_OUT_F32_ATOMIC_CONVW) {  // reference-layout scatter (rare path)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wc + 16 * j + l16;
        if (col >= p.N) continue;
        const float bv = add_bias ? p.bias[col] : 0.f;
        const int tap = col / p.convw_cin;
        const int ci = col - tap * p.convw_cin;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = m0 + wr + 16 * i + 4 * g4 + q;
          if (row < p.M) atomicAdd((float*)p.c + (long)row * p.ldc + ci * 9 + tap, p.alpha * acc[i][j][q] + bv);
        }
      }
    return;
  }
  float* p_c_slab = (float*)p.c;
  constexpr int SLD = BN + 4;
  static_assert(BM * SLD * 4 <= G::LDS_BYTES, "epilogue staging must fit the LDS allocation");
  float* sc = (float*)smem;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) sc[(wr + 16 * i + 4 * g4 + q) * SLD + wc + 16 * j + l16] = acc[i][j][q];
  __syncthreads();
  if (p.c_mode == ENCDIFF_OUT_F32_ATOMIC) {
    // lanes along columns: one wave instruction = 64 consecutive floats of one row
    for (int e = tid; e < BM * BN; e += 256) {
      const int r = e / BN, cc = e - r * BN;
      const int row = m0 + r, col = n0 + cc;
      if (row < p.M && col < p.N)
        atomicAdd((float*)p.c + (long)row * p.ldc + col, p.alpha * sc[r * SLD + cc] + (add_bias ? p.bias[col] : 0.f));
    }
    return;
  }
  if (p.split_k > 1 && p.c_mode == ENCDIFF_OUT_F32) {  // split-K slab of this z (workspace path)
    p_c_slab = (float*)p.c + (long)bz * p.M * p.N;
  }
  if (p.c_mode == ENCDIFF_OUT_BF16_GEGLU) {  // f (both halves) and y = value * gelu(gate)
    constexpr int H2 = BN / 2, CPH = H2 / 8;
    for (int e = tid; e < BM * CPH; e += 256) {
      const int r = e / CPH, c8 = (e - r * CPH) * 8, row = m0 + r;
      if (row >= p.M) continue;
      const int jv = gcol(c8), jg = gcol(c8 + H2);
      float a[8], g[8], y[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a[k] = p.alpha * sc[r * SLD + c8 + k] + (p.bias ? p.bias[jv + k] : 0.f);
        g[k] = p.alpha * sc[r * SLD + H2 + c8 + k] + (p.bias ? p.bias[jg + k] : 0.f);
      }
      bf16_t* F = (bf16_t*)p.c + (long)row * p.ldc;
      *(uint4*)(F + jv) = pack8(a);
      *(uint4*)(F + jg) = pack8(g);
#pragma unroll
      for (int k = 0; k < 8; ++k) y[k] = bf16_round(a[k]) * gelu_erf(bf16_round(g[k]));  // from the stored f
      *(uint4*)((bf16_t*)p.aux + (long)row * p.ld_aux + jv) = pack8(y);
    }
    return;
  }
  if (p.c_mode == ENCDIFF_OUT_BF16_GEGLU_BWD) {  // dy tile -> d(value), d(gate) from f
    constexpr int CPR = BN / 8;
    for (int e = tid; e < BM * CPR; e += 256) {
      const int r = e / CPR, c8 = (e - r * CPR) * 8;
      const int row = m0 + r, col = n0 + c8;
      if (row >= p.M || col >= p.N) continue;
      const bf16_t* F = (const bf16_t*)p.aux + (long)row * p.ld_aux;
      float a[8], g[8], da[8], dg[8];
      unpack8(*(const uint4*)(F + col), a);
      unpack8(*(const uint4*)(F + p.N + col), g);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = bf16_round(p.alpha * sc[r * SLD + c8 + k]);  // dy as the unfused path stores it
        da[k] = d * gelu_erf(g[k]);
        dg[k] = d * a[k] * gelu_erf_grad(g[k]);
      }
      bf16_t* D = (bf16_t*)p.c + (long)row * p.ldc;
      *(uint4*)(D + col) = pack8(da);
      *(uint4*)(D + p.N + col) = pack8(dg);
    }
    return;
  }
  // output row of GEMM row `row`: K4S2_TP rows are parity-major, each written to its pixel
  // (split-K slabs stay in GEMM row order; the finalize maps them)
  const bool slab_out = p.split_k > 1 && p.c == (void*)p.workspace;
  auto orow = [&](int row) -> long {
    if (md.k4 != 2 || slab_out) return row;
    const uint32_t mm = (uint32_t)row - mbase;
    const uint32_t b = fdiv(mm, aux.hw), r = mm - b * aux.hw.d;
    const uint32_t y = fdiv(r, aux.w), x = r - y * aux.w.d;
    return ((long)b * p.conv.h + 2 * y + (tp_q >> 1)) * p.conv.w + 2 * x + (tp_q & 1);
  };
  // in-kernel split-K combine: this split's slab goes out write-through (sc1)
  const bool fold = aux.fold.cnt != nullptr && slab_out;
  // (write-through stores for every slab measured slower in the step: 9.53 -> 9.64 ms, same box)
  const auto slab_rs = __builtin_amdgcn_make_buffer_rsrc(p.c, 0, fold ? p.split_k * p.M * p.N * 4 : 0, 0x00020000);
  const bool vec = (p.N % 8 == 0) && (p.ldc % 8 == 0) && (((uintptr_t)p.c & 15) == 0) &&
                   (!add_bias || (((uintptr_t)p.bias & 15) == 0)) &&
                   (!R || ((p.ld_resid % 8 == 0) && (((uintptr_t)R & 15) == 0)));
  if (vec) {
    constexpr int CPR = BN / 8;  // 8-column chunks per row
    for (int e = tid; e < BM * CPR; e += 256) {
      const int r = e / CPR, c8 = (e - r * CPR) * 8;
      const int row = m0 + r, col = n0 + c8;
      if (row >= p.M || col >= p.N) continue;
      const long ro = orow(row);
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = p.alpha * sc[r * SLD + c8 + k];
      if (add_bias) {
        const float4 b0 = *(const float4*)(p.bias + col), b1 = *(const float4*)(p.bias + col + 4);
        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
        v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
      }
      if (R) {
        float rr[8];
        unpack8(*(const uint4*)(R + ro * p.ld_resid + col), rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += rr[k];
      }
      if (p.c_mode == ENCDIFF_OUT_BF16) {
        const uint4 pk = pack8(v);
        *(uint4*)((bf16_t*)p.c + ro * p.ldc + col) = pk;
        if (p.gn_stats || p.ln_y) {  // the stored (bf16) values feed the statistics below
          float rv[8];
          unpack8(pk, rv);
#pragma unroll
          for (int k = 0; k < 8; ++k) sc[r * SLD + c8 + k] = rv[k];
        }
      } else {
        float* cp = p_c_slab + ro * p.ldc + col;
        if (p.c_mode == ENCDIFF_OUT_F32_ACCUM) {
          const float4 c0 = *(const float4*)cp, c1 = *(const float4*)(cp + 4);
          v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w;
          v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
        }
        if (fold) {  // write-through (sc1) slab stores: visible to the combining split without a release fence
          const int bo = (int)((cp - (const float*)p.c) * 4);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, make_float4(v[0], v[1], v[2], v[3])), slab_rs,
                                                 bo, 0, 16);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, make_float4(v[4], v[5], v[6], v[7])), slab_rs,
                                                 bo + 16, 0, 16);
        } else {
          *(float4*)cp = make_float4(v[0], v[1], v[2], v[3]);
          *(float4*)(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
  } else {
    for (int e = tid; e < BM * BN; e += 256) {
      const int r = e / BN, cc = e - r * BN;
      const int row = m0 + r, col = n0 + cc;
      if (row >= p.M || col >= p.N) continue;
      const long ro = orow(row);
      float v = p.alpha * sc[r * SLD + cc] + (add_bias ? p.bias[col] : 0.f);
      if (R) v += bf2f(R[ro * p.ld_resid + col]);
      if (p.c_mode == ENCDIFF_OUT_BF16) ((bf16_t*)p.c)[ro * p.ldc + col] = f2bf(v);
      else if (p.c_mode == ENCDIFF_OUT_F32_ACCUM) p_c_slab[ro * p.ldc + col] += v;
      else p_c_slab[ro * p.ldc + col] = v;
      if (p.gn_stats || p.ln_y) sc[r * SLD + cc] = bf16_round(v);
    }
  }
  if (fold) {
    // In-kernel split-K combine (the guide's write-through ticket recipe): every wave drains its
    // sc1 slab stores, then one lane takes the tile's ticket (relaxed, agent scope); the split that
    // draws split_k - 1 acquires and sums the tile's slabs in split order (bitwise reproducible,
    // placement independent), writes the user's output and leaves the ticket at zero.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)smem;  // the staging LDS is free: every thread is past its last read of it
    const int tile_id = by * ((p.M + BM - 1) / BM) + bx;
    if (tid == 0) {
      const int tk = __hip_atomic_fetch_add(aux.fold.cnt + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      flag[0] = tk == p.split_k - 1;
    }
    __syncthreads();
    if (!flag[0]) return;
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(aux.fold.cnt + tile_id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    const SplitFold& f = aux.fold;
    const long total = (long)p.M * p.N;
    constexpr int CPR = BN / 8;
    for (int e = tid; e < BM * CPR; e += 256) {
      const int r = e / CPR, c8 = (e - r * CPR) * 8;
      const int row = m0 + r, col = n0 + c8;
      if (row >= p.M || col >= p.N) continue;
      const float* s = (const float*)p.c + (long)row * p.N + col;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
      for (int z = 0; z < p.split_k; ++z) {
        const float4 a0 = *(const float4*)(s + z * total), a1 = *(const float4*)(s + z * total + 4);
        v[0] += a0.x; v[1] += a0.y; v[2] += a0.z; v[3] += a0.w;
        v[4] += a1.x; v[5] += a1.y; v[6] += a1.z; v[7] += a1.w;
      }
      {
        float bb[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (f.bias) {
          const float4 b0 = *(const float4*)(f.bias + col), b1 = *(const float4*)(f.bias + col + 4);
          bb[0] = b0.x; bb[1] = b0.y; bb[2] = b0.z; bb[3] = b0.w;
          bb[4] = b1.x; bb[5] = b1.y; bb[6] = b1.z; bb[7] = b1.w;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = splitk_scale(v[k], f.alpha, bb[k]);
      }
      if (f.resid) {
        float rr[8];
        unpack8(*(const uint4*)(f.resid + (long)row * f.ld_resid + col), rr);
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] += rr[k];
      }
      if (f.mode == ENCDIFF_OUT_BF16) {
        *(uint4*)((bf16_t*)f.c + (long)row * f.ldc + col) = pack8(v);
      } else {
        float* cp = (float*)f.c + (long)row * f.ldc + col;
        if (f.mode == ENCDIFF_OUT_F32_ACCUM) {
          const float4 c0 = *(const float4*)cp, c1 = *(const float4*)(cp + 4);
          v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w;
          v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
        }
        *(float4*)cp = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(cp + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    }
    return;
  }
  if (p.ln_y) {
    // LayerNorm of each produced row (host: n0 == 0 and N <= BN, OUT_BF16, split_k 1): TPR
    // adjacent lanes per row, mean then centred variance (two-pass, as the LayerNorm kernel),
    // from the stored bf16 values; normalised row written to ln_y.
    constexpr int TPR = 256 / BM;
    __syncthreads();
    const int r = tid / TPR, part = tid % TPR, row = m0 + r;
    const float* sr = sc + r * SLD;
    float sm = 0.f;
    for (int c8 = part * 8; c8 < p.N; c8 += TPR * 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) sm += sr[c8 + k];
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) sm += __shfl_xor(sm, o, 64);
    const float mean = sm / (float)p.N;
    float sq = 0.f;
    for (int c8 = part * 8; c8 < p.N; c8 += TPR * 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) { const float d = sr[c8 + k] - mean; sq += d * d; }
#pragma unroll
    for (int o = 1; o < TPR; o <<= 1) sq += __shfl_xor(sq, o, 64);
    const float rstd = rsqrtf(sq / (float)p.N + p.ln_eps);
    if (row < p.M) {
      if (part == 0) { p.ln_stats[2L * row] = mean; p.ln_stats[2L * row + 1] = rstd; }
      for (int c8 = part * 8; c8 < p.N; c8 += TPR * 8) {
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (sr[c8 + k] - mean) * rstd * p.ln_gamma[c8 + k] + p.ln_beta[c8 + k];
        *(uint4*)((bf16_t*)p.ln_y + (long)row * p.ld_ln_y + c8) = pack8(o);
      }
    }
  }
  if (p.gn_stats) {
    // GroupNorm statistics of the produced tensor (host: OUT_BF16, split_k 1, M % 64 == 0):
    // per 64-row segment and column, sum and sum of squares of the stored bf16 values.  Q row
    // phases per column, their partials added in phase order through LDS: deterministic.
    constexpr int Q = 256 / BN, NSEG = BM / 64;
    const int c = tid % BN, q = tid / BN;
    float ps[NSEG], pq[NSEG];
    __syncthreads();
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      float a = 0.f, b = 0.f;
#pragma unroll 4
      for (int r = sg * 64 + q; r < sg * 64 + 64; r += Q) {
        const float v = sc[r * SLD + c];
        a += v;
        b += v * v;
      }
      ps[sg] = a;
      pq[sg] = b;
    }
    __syncthreads();
    float* red = sc;  // [NSEG][2][Q][BN]
#pragma unroll
    for (int sg = 0; sg < NSEG; ++sg) {
      red[((sg * 2) * Q + q) * BN + c] = ps[sg];
      red[((sg * 2 + 1) * Q + q) * BN + c] = pq[sg];
    }
    __syncthreads();
    if (q == 0 && n0 + c < p.N) {
#pragma unroll
      for (int sg = 0; sg < NSEG; ++sg) {
        if (m0 + sg * 64 >= p.M) break;
        float a = 0.f, b = 0.f;
        for (int qq = 0; qq < Q; ++qq) {
          a += red[((sg * 2) * Q + qq) * BN + c];
          b += red[((sg * 2 + 1) * Q + qq) * BN + c];
        }
        const long slot = (m0 >> 6) + sg;
        p.gn_stats[(2 * slot) * p.ld_gn_stats + n0 + c] = a;
        p.gn_stats[(2 * slot + 1) * p.ld_gn_stats + n0 + c] = b;
      }
    }
  }
}

// Bijective XCD remap of a 1-D block id: the dispatcher deals workgroups round-robin over the 8
// XCDs (block b runs on XCD b % 8), so blocks b and b + 8 share an L2; the remap gives the blocks
// of one XCD CONSECUTIVE logical ids, i.e. neighbouring tiles: the same weight columns / k-slice
// (and, for implicit im2col, the neighbouring image rows the 3x3 taps reach) stay in one L2
// instead of being fetched by all eight.
ED_DEV int xcd_remap(int b, int n) {
  const int q = n >> 3, r = n & 7, x = b & 7;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
}

template <int BM, int BN, int AM, int BMD, int NS, int KB>
__global__ __launch_bounds__(256) void gemm_kernel(const EncdiffGemmArgs p, const GemmAux aux) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
  if (aux.xcd) {  // logical tile order x (M tiles) fastest, then y (N tiles), then z (k-slices)
    const int gx = gridDim.x, gy = gridDim.y;
    const int l = xcd_remap(bx + gx * (by + gy * bz), gx * gy * (int)gridDim.z);
    bx = l % gx;
    const int t = l / gx;
    by = t % gy;
    bz = t / gy;
  }
  gemm_tile<BM, BN, AM, BMD, NS, KB>(p, aux, bx, by, bz, smem);
}

__device__ __forceinline__ void gemm_finalize(const EncdiffGemmArgs& p, const int bid, const int nblk);

// Two independent GEMMs in one 1-D grid: blocks [0, n1) run problem 1 (64 x 64 tiles),
// the next n2 problem 2 (tile BM2 x BN2), the last nf the split-K finalize of an EARLIER
// launch's weight gradient (pf), deferred into this launch.  A layer's weight gradient
// (problem 1: deep split-K, the longer-running blocks, dispatched first) and its input
// gradient (problem 2) share the machine instead of running back to back, each too small
// to fill 256 CUs; the previous layer's weight-gradient finalize rides along, so neither
// needs a launch of its own.
template <int AM1, int BMD1, int BM2, int BN2, int AM2, int BMD2, int NS2, int KB2, int KB1, int NS1 = 2>
__global__ __launch_bounds__(256) void gemm2_kernel(const EncdiffGemmArgs p1, const GemmAux aux1,
                                                    const EncdiffGemmArgs p2, const GemmAux aux2, int gx1,
                                                    int gy1, int gx2, int gy2, const EncdiffGemmArgs pf, int nf) {
  extern __shared__ __attribute__((aligned(16))) bf16_t smem[];
  const int n1 = gx1 * gy1 * p1.split_k;
  const int n2 = gx2 * gy2 * p2.split_k;
  int i = blockIdx.x;
  if (i < n1) {
    // XCD of block i is i % 8 in both ranges (a rotation of the labels in the second): the remap
    // over each range keeps it bijective and XCD-grouped
    if (aux1.xcd) i = xcd_remap(i, n1);
    const int bx = i % gx1, t = i / gx1;
    gemm_tile<64, 64, AM1, BMD1, NS1, KB1>(p1, aux1, bx, t % gy1, t / gy1, smem);
  } else if (i < n1 + n2) {
    i -= n1;
    if (aux2.xcd) i = xcd_remap(i, n2);
    const int bx = i % gx2, t = i / gx2;
    gemm_tile<BM2, BN2, AM2, BMD2, NS2, KB2>(p2, aux2, bx, t % gy2, t / gy2, smem);
  } else {
    gemm_finalize(pf, i - n1 - n2, nf);
  }
}

// split-K finalize: C = alpha * sum_z slab[z] (+bias)(+resid).  Each lane owns 4
// consecutive outputs (float4 slab loads).  Up to 8 slabs one lane sums them all in z order
// (a workgroup covers 1024 outputs); deeper splits (e.g. 128 slabs of a 64x64 weight
// gradient) give 4 wave-rows every 4th slab and add the 4 partials in a fixed order.  Either
// way bitwise reproducible, no atomics.  The first version (one scalar load per lane,
// 64 outputs per workgroup) spent ~9 us on a 2048x256 split-4 GEMM in workgroup turnover.
constexpr int FIN_ZG = 4;
__host__ __device__ inline int fin_zgroups(const EncdiffGemmArgs& p) { return p.split_k > 8 ? FIN_ZG : 1; }
__host__ __device__ inline bool fin_vec(const EncdiffGemmArgs& p) {
  return (p.N & 3) == 0 && ((uintptr_t)p.workspace & 15) == 0;
}
// outputs one workgroup covers per grid-stride iteration
__host__ __device__ inline int fin_per_block(const EncdiffGemmArgs& p) {
  return (fin_vec(p) ? 4 : 1) * 256 / fin_zgroups(p);
}

// output row of GEMM row m (K4S2_TP: parity-major rows -> their pixel; plain division, the
// finalize is not on a hot path)
__device__ __forceinline__ long fin_row(const EncdiffGemmArgs& p, int m) {
  if (p.a_mode != ENCDIFF_OPA_IM2COL || p.conv.resample != ENCDIFF_RESAMPLE_K4S2_TP) return m;
  const int mq = p.M >> 2, q = m / mq, hh = p.conv.h >> 1, wh = p.conv.w >> 1;
  const int mm = m - q * mq, b = mm / (hh * wh), r = mm - b * hh * wh, y = r / wh, x = r - y * wh;
  return ((long)b * p.conv.h + 2 * y + (q >> 1)) * p.conv.w + 2 * x + (q & 1);
}

__device__ __forceinline__ void fin_store(const EncdiffGemmArgs& p, const bf16_t* R, const long i, float v) {
  const int row0 = (int)(i / p.N), col = (int)(i - (long)row0 * p.N);
  const long row = fin_row(p, row0);
  v = splitk_scale(v, p.alpha, p.bias ? p.bias[col] : 0.f);
  if (R) v += bf2f(R[(long)row * p.ld_resid + col]);
  if (p.c_mode == ENCDIFF_OUT_BF16) ((bf16_t*)p.c)[(long)row * p.ldc + col] = f2bf(v);
  else if (p.c_mode == ENCDIFF_OUT_F32_ACCUM) ((float*)p.c)[(long)row * p.ldc + col] += v;
  else ((float*)p.c)[(long)row * p.ldc + col] = v;
}

__device__ __forceinline__ void gemm_finalize(const EncdiffGemmArgs& p, const int bid, const int nblk) {
  // alpha / bias through splitk_scale: norm.hip's gn_slab_row restates this combine bitwise
  __shared__ float4 part[FIN_ZG][64];
  const long total = (long)p.M * p.N;
  const bf16_t* R = (const bf16_t*)p.resid;
  const int zgn = fin_zgroups(p);
  const int tpo = 256 / zgn;  // lanes per z-group
  const int o = threadIdx.x % tpo, zg = threadIdx.x / tpo;
  const long per = fin_per_block(p);
  if (fin_vec(p)) {
    for (long t0 = (long)bid * per; t0 < total; t0 += (long)nblk * per) {
      const long i = t0 + 4L * o;  // total % 4 == 0: the 4 outputs are in range together
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
      if (i < total) {
        const float* w = p.workspace + i;
#pragma unroll 8
        for (int z = zg; z < p.split_k; z += zgn) {
          const float4 v = *(const float4*)(w + (long)z * total);
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
      }
      if (zgn > 1) {  // block-uniform branch
        part[zg][o] = acc;
        __syncthreads();
        if (zg == 0) {
          const float4 a0 = part[0][o], a1 = part[1][o], a2 = part[2][o], a3 = part[3][o];
          acc.x = ((a0.x + a1.x) + a2.x) + a3.x;
          acc.y = ((a0.y + a1.y) + a2.y) + a3.y;
          acc.z = ((a0.z + a1.z) + a2.z) + a3.z;
          acc.w = ((a0.w + a1.w) + a2.w) + a3.w;
        }
      }
      if (zg == 0 && i < total) {
        // N % 4 == 0: one row.  32-bit division whenever the problem fits (uniform branch)
        const int row0 = total < (1L << 31) ? (int)i / p.N : (int)(i / p.N);
        const int col = (int)(i - (long)row0 * p.N);
        const long row = fin_row(p, row0);
        float v[4];
        {
          const float4 bb = p.bias ? make_float4(p.bias[col], p.bias[col + 1], p.bias[col + 2], p.bias[col + 3])
                                   : make_float4(0.f, 0.f, 0.f, 0.f);
          v[0] = splitk_scale(acc.x, p.alpha, bb.x);
          v[1] = splitk_scale(acc.y, p.alpha, bb.y);
          v[2] = splitk_scale(acc.z, p.alpha, bb.z);
          v[3] = splitk_scale(acc.w, p.alpha, bb.w);
        }
        if (R) {
#pragma unroll
          for (int k = 0; k < 4; ++k) v[k] += bf2f(R[(long)row * p.ld_resid + col + k]);
        }
        const long co = (long)row * p.ldc + col;
        if (p.c_mode == ENCDIFF_OUT_BF16) {
          bf16_t* c = (bf16_t*)p.c + co;
          if (((uintptr_t)c & 7) == 0) {  // one 8-byte store
            *(uint2*)c = make_uint2(pack2(v[0], v[1]), pack2(v[2], v[3]));
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) c[k] = f2bf(v[k]);
          }
        } else {
          float* c = (float*)p.c + co;
#pragma unroll
          for (int k = 0; k < 4; ++k) c[k] = p.c_mode == ENCDIFF_OUT_F32_ACCUM ? c[k] + v[k] : v[k];
        }
      }
      if (zgn > 1) __syncthreads();
    }
  } else {
    float* pz = (float*)part;
    for (long t0 = (long)bid * per; t0 < total; t0 += (long)nblk * per) {
      const long i = t0 + o;
      float acc = 0.f;
      if (i < total) {
        const float* w = p.workspace + i;
#pragma unroll 8
        for (int z = zg; z < p.split_k; z += zgn) acc += w[(long)z * total];
      }
      if (zgn > 1) {
        pz[zg * 64 + o] = acc;
        __syncthreads();
        if (zg == 0) acc = ((pz[o] + pz[64 + o]) + pz[128 + o]) + pz[192 + o];
      }
      if (zg == 0 && i < total) fin_store(p, R, i, acc);
      if (zgn > 1) __syncthreads();
    }
  }
  if (p.bias_grad) {  // bias-gradient slabs [split][M] behind the C slabs: 4 z-groups, fixed order
    float* pz = (float*)part;
    const int bo = threadIdx.x & 63, bz = threadIdx.x >> 6;
    const float* bs = p.workspace + (long)p.split_k * total;
    for (long t0 = (long)bid * 64; t0 < p.M; t0 += (long)nblk * 64) {
      const long m = t0 + bo;
      float acc = 0.f;
      if (m < p.M) {
#pragma unroll 8
        for (int z = bz; z < p.split_k; z += 4) acc += bs[(long)z * p.M + m];
      }
      __syncthreads();  // part may still be read by the C loop above
      pz[bz * 64 + bo] = acc;
      __syncthreads();
      if (bz == 0 && m < p.M) p.bias_grad[m] += ((pz[bo] + pz[64 + bo]) + pz[128 + bo]) + pz[192 + bo];
    }
  }
}

__global__ __launch_bounds__(256) void gemm_finalize_kernel(const EncdiffGemmArgs p) {
  gemm_finalize(p, blockIdx.x, gridDim.x);
}

// finalize of two split-K GEMMs in one launch (blocks [0, g1) for p1, the rest for p2)
__global__ __launch_bounds__(256) void gemm_finalize2_kernel(const EncdiffGemmArgs p1, const EncdiffGemmArgs p2,
                                                             int g1) {
  if ((int)blockIdx.x < g1) gemm_finalize(p1, blockIdx.x, g1);
  else gemm_finalize(p2, blockIdx.x - g1, gridDim.x - g1);
}

// ---------------------------------------------------------------------------
// 3x3 conv weight gradient, tile id 32 (WG3): dW[co][tap*cin + ci] += sum_p dY[p][co] x[p+tap][ci]
// (openaimodel_enc.py ResBlock / Upsample convs, autograd's weight gradient).
//
// The GEMM form (M = cout, N = 9 cin, K = pixels) stages every k-tile of dY once per 64 output
// columns and the im2col of x once per tap, and fills the chip only through deep split-K whose
// fp32 slabs are most of its HBM traffic.  Here a workgroup owns an output part of 32 couts x
// 16 cins x all 9 taps and a chunk of whole images; its 4 waves run independently over a
// quarter of the chunk each (no barrier in the main loop) and their partials are summed in LDS
// at the end, so a chunk writes ONE slab for 4x the pixels.  Per 32-pixel stage a wave stages
// dY (32 pixels x 32 couts, 2 KiB) and a zero-bordered halo of x (the stage's rows +-1, 16
// channels, 32 B per pixel slot) by LDS-DMA into its own ring; the B operand of tap (ty, tx)
// is the halo read at a constant offset (the ds_read immediate), so 9 taps cost 9 reads of one
// staged image instead of 9 staged im2col tiles.  18 MFMAs (2 cout tiles x 9 taps) per stage.
// k order within a stage: k = 8 g4 + 4 t + tq is pixel (img, y, x0 + tq) of the lane quad
// (g4, t) below, chosen so that the two 16-lane groups of each 32-lane half read halo rows
// (or images) whose slot distance is 4 mod 8: the transposed reads are bank-conflict free.
template <int W>
struct Wg3 {
  static constexpr int NI = W == 16 ? 1 : 2;                   // images per 32-pixel stage
  static constexpr int R = W == 4 ? 4 : 2;                     // image rows per stage
  static constexpr int WP = W == 16 ? 20 : (W == 8 ? 12 : 6);  // halo row pitch in pixel slots
  static constexpr int HR = R + 2;                             // halo rows per image
  static constexpr int NSLOT = NI * HR * WP;                   // halo pixel slots (32 B each)
  static constexpr int HCH = (2 * NSLOT + 63) / 64;            // halo LDS-DMA instructions (1 KiB)
  static constexpr int DYB = 32 * 64;                          // 32 k-rows x 32 couts (bf16)
  static constexpr int STAGE = DYB + HCH * 1024;               // bytes per ring stage
  static constexpr int LPS = 2 + HCH;                          // LDS-DMA instructions per stage
  static constexpr int T1 = W == 4 ? WP * 32 : 128;            // halo byte step of the lane's 2nd quad
  // lane quad (g4, t) of a stage -> (image, row, first column), stage-relative
  static ED_DEV void quad(int g4, int t, int& img, int& y, int& x0) {
    if constexpr (W == 16) { img = 0; y = g4 & 1; x0 = 8 * (g4 >> 1) + 4 * t; }
    else if constexpr (W == 8) { img = g4 >> 1; y = g4 & 1; x0 = 4 * t; }
    else { img = g4 & 1; y = 2 * (g4 >> 1) + t; x0 = 0; }
  }
};

// ds_read_b64_tr_b16 with an immediate byte offset (the tap / stage displacement)
template <int OFF>
ED_DEV v4s tr16_off(uint32_t a) {
  v4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(a), "i"(OFF));
  return r;
}
template <int N>
ED_DEV void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
ED_DEV v8bf cat8(v4s lo, v4s hi) {
  return __builtin_bit_cast(v8bf, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
// LDS byte address of a shared-memory pointer
ED_DEV uint32_t lds_addr(const void* p) {
  typedef __attribute__((address_space(3))) const char lds_char;
  return (uint32_t)(uintptr_t)(lds_char*)p;
}

template <int W, int NS>
struct Wg3Stage {
  // one 32-pixel stage in ring slot J: 2 cout tiles x 9 taps of MFMAs, reads software-pipelined
  // PD taps ahead with counted lgkmcnt waits (asm reads: hipcc does not track them)
  template <int J>
  static ED_DEV void compute(uint32_t a0, uint32_t a1, uint32_t bb, v4f (&acc)[2][9], bool bg, float (&bs)[2]) {
    using G = Wg3<W>;
    constexpr int SB = J * G::STAGE;
    constexpr int PD = 4;
    v8bf af0 = cat8(tr16_off<SB>(a0), tr16_off<SB + 256>(a0));
    v8bf af1 = cat8(tr16_off<SB>(a1), tr16_off<SB + 256>(a1));
    v8bf bf[9];
#define WG3_B(T) bf[T] = cat8(tr16_off<SB + G::DYB + ((T) / 3 * G::WP + (T) % 3) * 32>(bb), \
                              tr16_off<SB + G::DYB + ((T) / 3 * G::WP + (T) % 3) * 32 + G::T1>(bb))
    WG3_B(0); WG3_B(1); WG3_B(2); WG3_B(3);
#define WG3_T(T, NEXT, WAITN)                                                          \
    if constexpr ((NEXT) < 9) { WG3_B(NEXT); }                                         \
    lgkm_wait<WAITN>();                                                                \
    acc[0][T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af0, bf[T], acc[0][T], 0, 0, 0); \
    acc[1][T] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af1, bf[T], acc[1][T], 0, 0, 0);
    WG3_T(0, 4, 8) WG3_T(1, 5, 8) WG3_T(2, 6, 8) WG3_T(3, 7, 8) WG3_T(4, 8, 8)
    WG3_T(5, 9, 6) WG3_T(6, 9, 4) WG3_T(7, 9, 2) WG3_T(8, 9, 0)
#undef WG3_T
#undef WG3_B
    static_assert(PD == 4, "the wait counts above assume 4 taps in flight");
    if (bg) {  // bias gradient: this lane's 8 pixels of its cout in each tile
      const v8s s0 = __builtin_bit_cast(v8s, af0), s1 = __builtin_bit_cast(v8s, af1);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        bs[0] += bf2f((bf16_t)s0[e]);
        bs[1] += bf2f((bf16_t)s1[e]);
      }
    }
  }
};

// (the body is a __device__ function, as gemm_tile: a kernel template whose own body calls a lambda
// holding device builtins loses its host launch stub.  TAG: one body specialization per kernel --
// hipcc's host pass rejects a second kernel instantiation calling the same one)
// Split-K combine of a grouped weight gradient (wgrad_group_kernel; the SplitFold that wg_prepare
// sets): the workgroup's slab stores were write-through (sc1); after draining them, one lane takes
// the output part's ticket (relaxed, agent scope), and the chunk that draws split - 1 acquires and
// returns true -- it then sums the part's slabs in chunk order (bitwise reproducible, independent
// of which chunk arrives last or where it runs) -- and leaves the ticket at zero for the next launch.
// The guide's write-through ticket recipe, as the GEMM tiles' in-kernel combine.
ED_DEV bool wg_last_chunk(int* cnt, int split, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int tk = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = tk == split - 1;
  }
  __syncthreads();
  if (!flag[0]) return false;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return true;
}
constexpr int WG3_PART = 32 * 9 * 16, WGL_PART = 64 * 64;  // floats of one output part
ED_DEV float4 f4add(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
// the combined part written to the user's output: alpha, then += the output (F32_ACCUM)
ED_DEV void wg_fold_store(const SplitFold& f, float* o, float4 v) {
  v.x *= f.alpha; v.y *= f.alpha; v.z *= f.alpha; v.w *= f.alpha;
  if (f.mode == ENCDIFF_OUT_F32_ACCUM) v = f4add(v, *(const float4*)o);
  *(float4*)o = v;
}

template <int W, bool UP, int NS, int WPG, int TAG = 0>
__device__ __forceinline__ void wgrad3x3_body(const EncdiffGemmArgs& p, const int bid, char* wsm,
                                              const SplitFold* fold = nullptr) {
  using G = Wg3<W>;
  constexpr int H = W;
  constexpr uint32_t OOB = 0x80000000u;
  typedef __attribute__((address_space(3))) void lds_void;
  const int cin = p.conv.cin, cout = p.M;
  const int ncit = cin >> 4, nparts = (cout >> 5) * ncit;
  const int z = bid / nparts, part = bid - z * nparts;  // bid: the caller's logical block
  const int cot = part / ncit, cit = part - cot * ncit;
  const int co0 = cot * 32, ci0 = cit * 16;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l16 = lane & 15, g4 = lane >> 4, tq = l16 >> 2, tp = l16 & 3;
  const int ipz = p.conv.batch / p.split_k;               // images of this chunk
  const int nst = (ipz / G::NI) * (H / G::R) / WPG;      // 32-pixel stages of this wave
  const int st0 = wave * nst;                             // its first stage (chunk order)
  const int zb = z * ipz;
  char* ring = wsm + wave * (NS * G::STAGE);
  const uint32_t ring_a = lds_addr(ring);
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, 0, 0x7FFFFFF0, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, 0, 0x7FFFFFF0, 0x00020000);
  const uint32_t lda2 = (uint32_t)p.lda * 2u, ldx2 = (uint32_t)p.conv.ld_src * 2u;

  // staging invariants: dY chunk i (row r = k order, 16-B slot with the odd-8-row half swap)
  uint32_t dy_off[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = lane + 64 * i, r = c >> 2, gs = (c & 3) ^ (((r >> 3) & 1) << 1);
    int img, y, x0;
    G::quad(r >> 3, (r >> 2) & 1, img, y, x0);
    dy_off[i] = (uint32_t)((img * H + y) * W + x0 + (r & 3)) * lda2 + (uint32_t)(co0 + gs * 8) * 2u;
  }
  // halo chunk i: pixel slot s = c / 2, channel half c % 2
  int h_img[G::HCH], h_hy[G::HCH], h_xs[G::HCH];
  uint32_t h_ch[G::HCH];
#pragma unroll
  for (int i = 0; i < G::HCH; ++i) {
    const int c = lane + 64 * i, s = c >> 1;
    h_img[i] = s / (G::HR * G::WP);
    const int rem = s - h_img[i] * (G::HR * G::WP);
    h_hy[i] = rem / G::WP;
    const int hx = rem - h_hy[i] * G::WP;
    h_xs[i] = (s < G::NSLOT && hx >= 1 && hx <= W) ? hx - 1 : -1;  // -1: zero border / pad slot
    h_ch[i] = (uint32_t)(ci0 + (c & 1) * 8) * 2u;
  }
  auto stage = [&](int slot, int sw) {
    const int st = st0 + sw;
    const int b0 = zb + (st / (H / G::R)) * G::NI, y0 = (st % (H / G::R)) * G::R;
    char* sd = ring + slot * G::STAGE;
    const uint32_t pix0 = (uint32_t)(b0 * H + y0) * W;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(sd + i * 1024), 16, dy_off[i] + pix0 * lda2, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < G::HCH; ++i) {
      const int ys = y0 + h_hy[i] - 1, xs = h_xs[i];
      const bool ok = xs >= 0 && (unsigned)ys < (unsigned)H;
      const uint32_t b = (uint32_t)(b0 + h_img[i]);
      const uint32_t sp = UP ? (b * (H / 2) + (uint32_t)(ys >> 1)) * (W / 2) + (uint32_t)(xs >> 1)
                             : (b * H + (uint32_t)ys) * W + (uint32_t)xs;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void*)(sd + G::DYB + i * 1024), 16, ok ? sp * ldx2 + h_ch[i] : OOB,
                                               0, 0, 0);
    }
  };
  // fragment read bases (ring slot 0; the slot offset is the reads' immediate)
  const uint32_t a0 = ring_a + (uint32_t)((g4 * 8 + tq) * 64 + ((0 ^ (g4 & 1)) * 32) + tp * 8);
  const uint32_t a1 = ring_a + (uint32_t)((g4 * 8 + tq) * 64 + ((1 ^ (g4 & 1)) * 32) + tp * 8);
  uint32_t bb;
  {
    int img, y, x0;
    G::quad(g4, 0, img, y, x0);
    bb = ring_a + (uint32_t)(((img * G::HR + y) * G::WP + x0 + tq) * 32 + tp * 8);
  }
  v4f acc[2][9];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[m][t] = (v4f){0.f, 0.f, 0.f, 0.f};
  const bool bg = p.bias_grad != nullptr && cit == 0;
  float bs[2] = {0.f, 0.f};

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nst) stage(s, s);
  for (int s0 = 0; s0 < nst; s0 += NS) {
#define WG3_IT(J)                                                                              \
    if (s0 + (J) < nst) {                                                                      \
      const int s = s0 + (J);                                                                  \
      if (s + NS - 1 < nst) { vm_wait<G::LPS * (NS - 2)>(); }                                  \
      else { vm_wait_stages<G::LPS, NS - 2>(nst - 1 - s); }                                    \
      if (s + NS - 1 < nst) stage(((J) + NS - 1) % NS, s + NS - 1);                           \
      Wg3Stage<W, NS>::template compute<J>(a0, a1, bb, acc, bg, bs);                           \
    }
    WG3_IT(0)
    WG3_IT(1)
    if constexpr (NS > 2) { WG3_IT(2) }
    if constexpr (NS > 3) { WG3_IT(3) }
    if constexpr (NS > 4) { WG3_IT(4) }
    if constexpr (NS > 5) { WG3_IT(5) }
    if constexpr (NS > 6) { WG3_IT(6) }
    static_assert(NS <= 7, "ring slots are unrolled up to 7");
#undef WG3_IT
  }

  // ---- epilogue, one cout tile (16 couts) at a time so the LDS image stays <= the ring: every
  // wave parks its partial [16 co][9 tap][16 ci] in LDS, then all threads sum the WPG partials in
  // wave order (fixed: reproducible) over float4 runs of 4 cins and store them 16 B per lane --
  // into this chunk's slab write-through (sc1: measured 1 us faster than write-back slabs, whose
  // dirty lines the end of the kernel flushes), or into C itself without split-K ----
  constexpr int HALF = 16 * 9 * 16;
  float* red = (float*)wsm;             // [WPG][HALF]
  float* bred = red + WPG * HALF;       // [WPG][32] bias partials
  const bool slab = p.split_k > 1;
  const long MN = (long)p.M * p.N;
  float* out = (float*)p.c + (slab ? (long)z * MN : 0);
  const long ldo = slab ? p.N : p.ldc;
  const auto rso = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, 0x7FFFFFF0, 0x00020000);
  const auto rsp = __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    __syncthreads();  // ring (m = 0) / the previous half's image (m = 1) no longer read
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) red[wave * HALF + ((4 * g4 + q) * 9 + t) * 16 + l16] = acc[m][t][q];
    if (m == 0 && bg) {
#pragma unroll
      for (int mm = 0; mm < 2; ++mm) {
        float v = bs[mm];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) bred[wave * 32 + mm * 16 + lane] = v;
      }
    }
    __syncthreads();
    for (int f = threadIdx.x; f < HALF / 4; f += WPG * 64) {
      float4 v = *(const float4*)(red + 4 * f);
#pragma unroll
      for (int w = 1; w < WPG; ++w) {
        const float4 u = *(const float4*)(red + w * HALF + 4 * f);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
      }
      const int c4 = f & 3, ct = f >> 2, t = ct % 9, co = co0 + m * 16 + ct / 9;
      const long off = (long)co * ldo + t * cin + ci0 + 4 * c4;
      if (slab && fold) {  // part-major slab [z][part][32 co][9 tap][16 ci]: no cache line shared by two parts
        const long po = ((long)z * nparts + part) * WG3_PART + (m * 16 + ct / 9) * 144 + t * 16 + 4 * c4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rsp, (int)(po * 4), 0, 16);
      } else if (slab) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rso, (int)(off * 4), 0, 16);
      } else {
        float4* o = (float4*)(out + off);
        v.x *= p.alpha; v.y *= p.alpha; v.z *= p.alpha; v.w *= p.alpha;
        if (p.c_mode == ENCDIFF_OUT_F32_ACCUM) {
          const float4 c = *o;
          v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
        }
        *o = v;
      }
    }
  }
  if (bg && threadIdx.x < 32) {
    float v = bred[threadIdx.x];
#pragma unroll
    for (int w = 1; w < WPG; ++w) v += bred[w * 32 + threadIdx.x];
    const int co = co0 + threadIdx.x;
    if (slab && fold) {  // write-through, as the slab, at [cout tile][z][32]: read by the combining chunk
      const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.workspace, 0, 0x7FFFFFF0, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(
          __builtin_bit_cast(uint32_t, v), rsw,
          (int)(((long)p.split_k * MN + ((long)cot * p.split_k + z) * 32 + threadIdx.x) * 4), 0, 16);
    } else if (slab) {
      p.workspace[(long)p.split_k * MN + (long)z * p.M + co] = v;
    } else {
      p.bias_grad[co] += v;
    }
  }
  if (!(slab && fold) || !wg_last_chunk(fold->cnt + part, p.split_k, (int*)wsm)) return;
  // the combining chunk: the part's [32 co][9 tap][16 ci] summed over the chunks in order
  const float* s0 = (const float*)p.c + (long)part * WG3_PART;
  const long zs = (long)nparts * WG3_PART;
  for (int f = threadIdx.x; f < 32 * 9 * 4; f += WPG * 64) {
    const int cl = f / 36, r = f % 36, t = r >> 2, c4 = r & 3;
    const int lo = cl * 144 + t * 16 + 4 * c4;
    float4 v = *(const float4*)(s0 + lo);
    for (int zz = 1; zz < p.split_k; ++zz) v = f4add(v, *(const float4*)(s0 + zz * zs + lo));
    wg_fold_store(*fold, (float*)fold->c + (long)(co0 + cl) * fold->ldc + t * cin + ci0 + 4 * c4, v);
  }
  if (bg && threadIdx.x < 32) {
    const float* bz = p.workspace + (long)p.split_k * MN + (long)cot * p.split_k * 32 + threadIdx.x;
    float v = bz[0];
    for (int zz = 1; zz < p.split_k; ++zz) v += bz[zz * 32];
    p.bias_grad[co0 + threadIdx.x] += v;
  }
}

// The WG3 grid: blocks [0, nblk) the weight gradient, then (BM2 > 0) the layer's input-gradient
// GEMM tiles in the same grid (as gemm2_kernel pairs two GEMM tiles: each alone leaves most of the
// chip idle), then a deferred finalize of an earlier weight gradient riding along.
template <int W, bool UP, int NS, int WPG, int BM2 = 0, int BN2 = 0, int AM2 = 0, int BMD2 = 0, int NS2 = 0>
__global__ __launch_bounds__(WPG * 64) void wgrad3x3_kernel(const EncdiffGemmArgs p, int nblk, const EncdiffGemmArgs pf,
                                                            int nf, const EncdiffGemmArgs p2, const GemmAux aux2, int gx2,
                                                            int gy2) {
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  int i = blockIdx.x;
  if (i < nblk) {
    // a chunk's parts (sharing dY / x rows) on one XCD
    wgrad3x3_body<W, UP, NS, WPG, BM2 * 1000 + BN2 * 10 + AM2>(p, xcd_remap(i, nblk), wsm);
    return;
  }
  i -= nblk;
  if constexpr (BM2 > 0) {
    const int n2 = gx2 * gy2 * p2.split_k;
    if (i < n2) {
      const int bx = i % gx2, t = i / gx2;
      gemm_tile<BM2, BN2, AM2, BMD2, NS2, BK>(p2, aux2, bx, t % gy2, t / gy2, (bf16_t*)wsm);
      return;
    }
    i -= n2;
  }
  // finalize blocks (4-wave grids only: wg3_launch launches a tile-33 grid's finalize on its own)
  if (WPG != 4) return;
  gemm_finalize(pf, i, nf);
}

// tile 32: 4 waves per workgroup, paired with the layer's input gradient in one grid where the pair
// path allows; 34: 4 waves, never paired; 33: 8 waves (two per SIMD on one workgroup per CU), never
// paired; 3-deep stage rings alone, 2-deep paired
template <int W, int NS, int WPG>
constexpr size_t wg3_lds() {
  constexpr size_t ring = WPG * NS * Wg3<W>::STAGE, red = (WPG * 16 * 9 * 16 + WPG * 32) * 4;
  return ring > red ? ring : red;
}
__host__ __device__ constexpr int wg3_waves(int tile) { return tile == 33 ? 8 : 4; }
constexpr int WG3_PAIR_NS = 2;  // paired launch: 2-deep rings keep the shared LDS size small

// ---------------------------------------------------------------------------
// Linear weight gradient, tile id 36 (WGL): dW[m][n] += sum_t dY[t][m] x[t][n] over T tokens
// (every nn.Linear / 1x1 conv of the UNet: attention.py proj_in/out, to_q/k/v/out, ff; the
// ResBlock skip).  Small output, long K: as WG3, a workgroup owns a 64 x 64 output part and a
// chunk of tokens, its 4 waves run independently over a quarter of the chunk each (32-token
// stages: dY and x rows, 4 KiB each, staged by LDS-DMA into the wave's own ring; 4 x 4 MFMA tiles
// per stage) and their partials are summed in LDS: one slab per chunk.  Rows are 128 B (64
// bf16); the 32-B column groups a transposed read touches are XOR-swizzled by row bits 1 and 3
// so both 16-lane groups of a 32-lane half hit distinct banks.
struct Wgl {
  static constexpr int ROWB = 128;               // 64 columns x bf16
  static constexpr int OPB = 32 * ROWB;          // one operand of a 32-token stage (4 KiB)
  static constexpr int STAGE = 2 * OPB;          // dY rows then x rows
  static constexpr int LPS = 8;                  // LDS-DMA instructions per stage
  // 16-B slot of global chunk gc (0..7) in row r
  static ED_DEV int slot(int r, int gc) { return ((((gc >> 1) ^ ((r >> 1) & 1) ^ (((r >> 3) & 1) << 1))) << 1) | (gc & 1); }
};

template <int NS>
struct WglStage {
  template <int J>
  static ED_DEV void compute(const uint32_t (&ab)[4], const uint32_t (&bb)[4], v4f (&acc)[4][4], bool bg, float (&bs)[4]) {
    constexpr int SB = J * Wgl::STAGE;
    v8bf af[4], bf[4];
#define WGL_RD(F, BASE, I, OFF) F[I] = cat8(tr16_off<SB + (OFF)>(BASE[I]), tr16_off<SB + (OFF) + 4 * Wgl::ROWB>(BASE[I]))
    WGL_RD(af, ab, 0, 0); WGL_RD(af, ab, 1, 0); WGL_RD(af, ab, 2, 0); WGL_RD(af, ab, 3, 0);
    WGL_RD(bf, bb, 0, Wgl::OPB); WGL_RD(bf, bb, 1, Wgl::OPB);
    WGL_RD(bf, bb, 2, Wgl::OPB); WGL_RD(bf, bb, 3, Wgl::OPB);
    lgkm_wait<4>();  // A and B tiles 0, 1 landed (tiles 2, 3 = the 4 youngest reads)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[0], acc[i][0], 0, 0, 0);
      acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[1], acc[i][1], 0, 0, 0);
    }
    lgkm_wait<0>();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i][2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[2], acc[i][2], 0, 0, 0);
      acc[i][3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[3], acc[i][3], 0, 0, 0);
    }
#undef WGL_RD
    if (bg) {  // bias gradient: this lane's 8 tokens of its output column in each m tile
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const v8s sv = __builtin_bit_cast(v8s, af[i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) bs[i] += bf2f((bf16_t)sv[e]);
      }
    }
  }
};

template <int NS, int TAG = 0>
__device__ __forceinline__ void wgradlin_body(const EncdiffGemmArgs& p, const int bid, char* wsm,
                                              const SplitFold* fold = nullptr) {
  typedef __attribute__((address_space(3))) void lds_void;
  const int ntn = p.N >> 6, nparts = (p.M >> 6) * ntn;
  const int z = bid / nparts, part = bid - z * nparts;  // bid: the caller's logical block
  const int mt = part / ntn, nt = part - mt * ntn;
  const int m0 = mt * 64, n0 = nt * 64;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int l16 = lane & 15, g4 = lane >> 4, tq = l16 >> 2, tp = l16 & 3;
  const int tpz = p.K / p.split_k;        // tokens of this chunk
  const int nst = tpz / (32 * 4);         // 32-token stages of this wave
  const int t0 = z * tpz + wave * nst * 32;
  char* ring = wsm + wave * (NS * Wgl::STAGE);
  const uint32_t ring_a = lds_addr(ring);
  const auto rsA = __builtin_amdgcn_make_buffer_rsrc((void*)p.a, 0, 0x7FFFFFF0, 0x00020000);
  const auto rsB = __builtin_amdgcn_make_buffer_rsrc((void*)p.b, 0, 0x7FFFFFF0, 0x00020000);
  const uint32_t lda2 = (uint32_t)p.lda * 2u, ldb2 = (uint32_t)p.ldb * 2u;
  // staging: LDS chunk c = lane + 64 i of an operand -> row r = c / 8, slot c % 8 holds global chunk gc
  uint32_t a_off[4], b_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = lane + 64 * i, r = c >> 3, sl = c & 7;
    int gc = 0;
#pragma unroll
    for (int g = 0; g < 8; ++g)
      if (Wgl::slot(r, g) == sl) gc = g;
    a_off[i] = (uint32_t)r * lda2 + (uint32_t)(m0 + gc * 8) * 2u;
    b_off[i] = (uint32_t)r * ldb2 + (uint32_t)(n0 + gc * 8) * 2u;
  }
  auto stage = [&](int slot, int sw) {
    char* sd = ring + slot * Wgl::STAGE;
    const uint32_t row0 = (uint32_t)(t0 + sw * 32);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_void*)(sd + i * 1024), 16, a_off[i] + row0 * lda2, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_void*)(sd + Wgl::OPB + i * 1024), 16, b_off[i] + row0 * ldb2, 0,
                                               0, 0);
  };
  // fragment bases (ring slot 0, first 4 rows of the lane's k group): column tile i at row r
  uint32_t ab[4], bb[4];
  {
    const int r = g4 * 8 + tq;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gc = 2 * i + (tp >> 1);  // 16-B chunk of columns 16 i + 4 tp .. + 3
      const uint32_t o = (uint32_t)(r * Wgl::ROWB + Wgl::slot(r, gc) * 16 + (tp & 1) * 8);
      ab[i] = ring_a + o;
      bb[i] = ring_a + o;
    }
  }
  // (rows r and r + 4 differ in bit 2 only: same swizzle, the second read is 4 rows on)
  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  const bool bg = p.bias_grad != nullptr && nt == 0;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nst) stage(s, s);
  for (int s0 = 0; s0 < nst; s0 += NS) {
#define WGL_IT(J)                                                                              \
    if (s0 + (J) < nst) {                                                                      \
      const int s = s0 + (J);                                                                  \
      if (s + NS - 1 < nst) { vm_wait<Wgl::LPS * (NS - 2)>(); }                                \
      else { vm_wait_stages<Wgl::LPS, NS - 2>(nst - 1 - s); }                                  \
      if (s + NS - 1 < nst) stage(((J) + NS - 1) % NS, s + NS - 1);                           \
      WglStage<NS>::template compute<J>(ab, bb, acc, bg, bs);                                  \
    }
    WGL_IT(0)
    WGL_IT(1)
    if constexpr (NS > 2) { WGL_IT(2) }
    if constexpr (NS > 3) { WGL_IT(3) }
    static_assert(NS <= 4, "ring slots are unrolled up to 4");
#undef WGL_IT
  }
  // ---- epilogue (as WG3's): 32 output rows at a time through LDS, partials summed in wave order
  constexpr int HALF = 32 * 64;
  float* red = (float*)wsm;        // [4][HALF]
  float* bred = red + 4 * HALF;    // [4][64]
  const bool slab = p.split_k > 1;
  const long MN = (long)p.M * p.N;
  float* out = (float*)p.c + (slab ? (long)z * MN : 0);
  const long ldo = slab ? p.N : p.ldc;
  const auto rso = __builtin_amdgcn_make_buffer_rsrc((void*)out, 0, 0x7FFFFFF0, 0x00020000);
  const auto rsp = __builtin_amdgcn_make_buffer_rsrc((void*)p.c, 0, 0x7FFFFFF0, 0x00020000);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) red[wave * HALF + (i * 16 + 4 * g4 + q) * 64 + j * 16 + l16] = acc[2 * h + i][j][q];
    if (h == 0 && bg) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = bs[i];
        v += __shfl_xor(v, 16, 64);
        v += __shfl_xor(v, 32, 64);
        if (lane < 16) bred[wave * 64 + i * 16 + lane] = v;
      }
    }
    __syncthreads();
    for (int f = threadIdx.x; f < HALF / 4; f += 256) {
      float4 v = *(const float4*)(red + 4 * f);
#pragma unroll
      for (int w = 1; w < 4; ++w) {
        const float4 u = *(const float4*)(red + w * HALF + 4 * f);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
      }
      const int row = m0 + h * 32 + (f >> 4), col = n0 + 4 * (f & 15);
      const long off = (long)row * ldo + col;
      if (slab && fold) {  // part-major slab [z][part][64][64]: no cache line shared by two parts
        const long po = ((long)z * nparts + part) * WGL_PART + (h * 32 + (f >> 4)) * 64 + 4 * (f & 15);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rsp, (int)(po * 4), 0, 16);
      } else if (slab) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32, v), rso, (int)(off * 4), 0, 16);
      } else {
        float4* o = (float4*)(out + off);
        v.x *= p.alpha; v.y *= p.alpha; v.z *= p.alpha; v.w *= p.alpha;
        if (p.c_mode == ENCDIFF_OUT_F32_ACCUM) {
          const float4 c = *o;
          v.x += c.x; v.y += c.y; v.z += c.z; v.w += c.w;
        }
        *o = v;
      }
    }
  }
  if (bg && threadIdx.x < 64) {
    float v = bred[threadIdx.x];
#pragma unroll
    for (int w = 1; w < 4; ++w) v += bred[w * 64 + threadIdx.x];
    const int m = m0 + threadIdx.x;
    if (slab && fold) {  // write-through, as the slab, at [row tile][z][64]: read by the combining chunk
      const auto rsw = __builtin_amdgcn_make_buffer_rsrc((void*)p.workspace, 0, 0x7FFFFFF0, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b32(
          __builtin_bit_cast(uint32_t, v), rsw,
          (int)(((long)p.split_k * MN + ((long)mt * p.split_k + z) * 64 + threadIdx.x) * 4), 0, 16);
    } else if (slab) {
      p.workspace[(long)p.split_k * MN + (long)z * p.M + m] = v;
    } else {
      p.bias_grad[m] += v;
    }
  }
  if (!(slab && fold) || !wg_last_chunk(fold->cnt + part, p.split_k, (int*)wsm)) return;
  // the combining chunk: the 64 x 64 part summed over the chunks in order, 16 B per lane
  const float* s0 = (const float*)p.c + (long)part * WGL_PART;
  const long zs = (long)nparts * WGL_PART;
  for (int f = threadIdx.x; f < 64 * 16; f += 256) {
    const int lo = (f >> 4) * 64 + 4 * (f & 15);
    float4 v = *(const float4*)(s0 + lo);
    for (int zz = 1; zz < p.split_k; ++zz) v = f4add(v, *(const float4*)(s0 + zz * zs + lo));
    wg_fold_store(*fold, (float*)fold->c + (long)(m0 + (f >> 4)) * fold->ldc + n0 + 4 * (f & 15), v);
  }
  if (bg && threadIdx.x < 64) {
    const float* bz = p.workspace + (long)p.split_k * MN + (long)mt * p.split_k * 64 + threadIdx.x;
    float v = bz[0];
    for (int zz = 1; zz < p.split_k; ++zz) v += bz[zz * 64];
    p.bias_grad[m0 + threadIdx.x] += v;
  }
}

// The WGL grid: [0, nblk) the weight gradient, then (BM2 > 0) the layer's input-gradient GEMM tiles,
// then a deferred finalize riding along
template <int NS, int BM2 = 0, int BN2 = 0, int AM2 = 0, int BMD2 = 0, int NS2 = 0, int KB2 = BK>
__global__ __launch_bounds__(256) void wgradlin_kernel(const EncdiffGemmArgs p, int nblk, const EncdiffGemmArgs pf, int nf,
                                                       const EncdiffGemmArgs p2, const GemmAux aux2, int gx2, int gy2) {
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  int i = blockIdx.x;
  if (i < nblk) {
    // a chunk's parts (sharing dY / x rows) on one XCD
    wgradlin_body<NS, BM2 * 100000 + BN2 * 100 + NS2 * 10 + (KB2 == BK ? 0 : 1)>(p, xcd_remap(i, nblk), wsm);
    return;
  }
  i -= nblk;
  if constexpr (BM2 > 0) {
    const int n2 = gx2 * gy2 * p2.split_k;
    if (i < n2) {
      const int bx = i % gx2, t = i / gx2;
      gemm_tile<BM2, BN2, AM2, BMD2, NS2, KB2>(p2, aux2, bx, t % gy2, t / gy2, (bf16_t*)wsm);
      return;
    }
    i -= n2;
  }
  gemm_finalize(pf, i, nf);
}

constexpr int WGL_NS = 3, WGL_PAIR_NS = 2;
template <int NS>
constexpr size_t wgl_lds() {
  constexpr size_t ring = 4 * NS * Wgl::STAGE, red = (4 * 32 * 64 + 4 * 64) * 4;
  return ring > red ? ring : red;
}

int wgl_check(const EncdiffGemmArgs& p) {
  if (p.a_mode != ENCDIFF_OPA_ROWM || p.b_mode != ENCDIFF_OPB_ROWN) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.c_mode != ENCDIFF_OUT_F32 && p.c_mode != ENCDIFF_OUT_F32_ACCUM) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.M % 64 || p.N % 64 || p.split_k < 1 || p.K % (p.split_k * 128)) return ENCDIFF_ERR_SHAPE;
  if (p.lda % 8 || p.ldb % 8 || ((uintptr_t)p.a & 15) || ((uintptr_t)p.b & 15)) return ENCDIFF_ERR_SHAPE;
  if (p.split_k > 1 ? ((uintptr_t)p.workspace & 15) != 0 : (p.ldc % 4 || ((uintptr_t)p.c & 15))) return ENCDIFF_ERR_SHAPE;
  return ENCDIFF_OK;
}

hipError_t wgl_launch(const EncdiffGemmArgs& p, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  constexpr size_t lds = wgl_lds<WGL_NS>();
  static const hipError_t attr_ok =
      hipFuncSetAttribute((const void*)wgradlin_kernel<WGL_NS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr_ok != hipSuccess) return attr_ok;
  const int nblk = (p.M / 64) * (p.N / 64) * p.split_k;
  hipLaunchKernelGGL((wgradlin_kernel<WGL_NS>), dim3((unsigned)(nblk + nf)), dim3(256), lds, s, p, nblk, pf, nf, p,
                     GemmAux{}, 0, 0);
  return hipGetLastError();
}

// eligibility of a prepared weight-gradient plan for the WG3 kernel
int wg3_check(const EncdiffGemmArgs& p) {
  const EncdiffConvGeom& g = p.conv;
  if (p.a_mode != ENCDIFF_OPA_ROWM || p.b_mode != ENCDIFF_OPB_IM2COL) return ENCDIFF_ERR_UNSUPPORTED;
  if (g.resample != ENCDIFF_RESAMPLE_NONE && g.resample != ENCDIFF_RESAMPLE_UP2) return ENCDIFF_ERR_UNSUPPORTED;
  if (g.h != g.w || (g.w != 4 && g.w != 8 && g.w != 16)) return ENCDIFF_ERR_UNSUPPORTED;
  if (p.M % 32 || g.cin % 16 || p.N != 9 * g.cin || (long)p.K != (long)g.batch * g.h * g.w) return ENCDIFF_ERR_SHAPE;
  if (p.c_mode != ENCDIFF_OUT_F32 && p.c_mode != ENCDIFF_OUT_F32_ACCUM) return ENCDIFF_ERR_UNSUPPORTED;
  const int ni = g.w == 16 ? 1 : 2, rows = g.w == 4 ? 4 : 2;
  if (p.split_k < 1 || g.batch % p.split_k || (g.batch / p.split_k) % ni) return ENCDIFF_ERR_SHAPE;
  const int nst = (g.batch / p.split_k / ni) * (g.h / rows);  // 32-pixel stages per chunk
  if (nst % wg3_waves(p.tile)) return ENCDIFF_ERR_SHAPE;
  if (p.lda % 8 || g.ld_src % 8 || ((uintptr_t)p.a & 15) || ((uintptr_t)p.b & 15)) return ENCDIFF_ERR_SHAPE;
  // float4 epilogue stores: slabs or C itself 16-byte aligned
  if (p.split_k > 1 ? ((uintptr_t)p.workspace & 15) != 0 : (p.ldc % 4 || ((uintptr_t)p.c & 15))) return ENCDIFF_ERR_SHAPE;
  return ENCDIFF_OK;
}

template <int W, bool UP, int NS, int WPG>
hipError_t wg3_launch_t(const EncdiffGemmArgs& p, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  constexpr size_t lds = wg3_lds<W, NS, WPG>();
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)wgrad3x3_kernel<W, UP, NS, WPG>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr_ok != hipSuccess) return attr_ok;
  const int nblk = (p.M / 32) * (p.conv.cin / 16) * p.split_k;
  hipLaunchKernelGGL((wgrad3x3_kernel<W, UP, NS, WPG>), dim3((unsigned)(nblk + nf)), dim3(WPG * 64), lds, s, p, nblk, pf,
                     nf, p, GemmAux{}, 0, 0);
  return hipGetLastError();
}

template <int WPG>
hipError_t wg3_launch_w(const EncdiffGemmArgs& p, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  const bool up = p.conv.resample == ENCDIFF_RESAMPLE_UP2;
  switch (p.conv.w) {
    case 4: return up ? wg3_launch_t<4, true, 3, WPG>(p, pf, nf, s) : wg3_launch_t<4, false, 3, WPG>(p, pf, nf, s);
    case 8: return up ? wg3_launch_t<8, true, 3, WPG>(p, pf, nf, s) : wg3_launch_t<8, false, 3, WPG>(p, pf, nf, s);
    default: return up ? wg3_launch_t<16, true, 3, WPG>(p, pf, nf, s) : wg3_launch_t<16, false, 3, WPG>(p, pf, nf, s);
  }
}

hipError_t wg3_launch(const EncdiffGemmArgs& p, int tile, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  if (tile == 33) {
    // 8-wave workgroups: a riding finalize would reach gemm_finalize's barriers after waves 4-7
    // returned (a barrier after a divergent exit) -- run it as a launch of its own instead
    if (nf > 0) {
      hipLaunchKernelGGL(gemm_finalize_kernel, dim3((unsigned)nf), dim3(256), 0, s, pf);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return wg3_launch_w<8>(p, pf, 0, s);
  }
  return wg3_launch_w<4>(p, pf, nf, s);
}

template <int BM, int BN, int AM, int BMD, int NS = 2, int KB = BK>
hipError_t launch_t(const EncdiffGemmArgs& p, const GemmAux& aux, hipStream_t s) {
  using G = Gemm<BM, BN, AM, BMD, NS, KB>;
  const size_t lds = G::LDS_BYTES;
  // dynamic LDS above 64 KiB must be opted in once per instantiation (thread-safe static init)
  static const hipError_t attr_ok = hipFuncSetAttribute(
      (const void*)gemm_kernel<BM, BN, AM, BMD, NS, KB>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr_ok != hipSuccess) return attr_ok;
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, p.split_k);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, AM, BMD, NS, KB>), grid, dim3(256), lds, s, p, aux);
  return hipGetLastError();
}

// GroupNorm-in-staging forward conv (EncdiffGemmArgs.agn_*): 64x64 tiles, 2-deep ring, the
// per-(image, channel) coefficient table behind the ring in dynamic LDS
hipError_t launch_agn(const EncdiffGemmArgs& p, const GemmAux& aux, hipStream_t s) {
  using G = Gemm<64, 64, A_IM2COL_GN, B_ROWK, 2, BK>;
  const int hw = p.conv.h * p.conv.w;
  const int nimg = (63 / hw + 2) < p.conv.batch ? 63 / hw + 2 : p.conv.batch;  // images one 64-row tile reads
  const size_t lds = (size_t)G::LDS_BYTES + (size_t)nimg * p.conv.cin * 8;
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)gemm_kernel<64, 64, A_IM2COL_GN, B_ROWK, 2, BK>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
  if (attr_ok != hipSuccess) return attr_ok;
  if (lds > 156 * 1024) return hipErrorInvalidValue;
  dim3 grid((p.M + 63) / 64, (p.N + 63) / 64, p.split_k);
  hipLaunchKernelGGL((gemm_kernel<64, 64, A_IM2COL_GN, B_ROWK, 2, BK>), grid, dim3(256), lds, s, p, aux);
  return hipGetLastError();
}

// LayerNorm-in-staging linear (EncdiffGemmArgs.lna_*): 64x64 tiles, 2-deep ring, row statistics
// and gamma / beta behind the ring in dynamic LDS
hipError_t launch_lna(const EncdiffGemmArgs& p, const GemmAux& aux, hipStream_t s) {
  using G = Gemm<64, 64, A_ROWK_LN, B_ROWK, 2, BK>;
  const size_t lds = (size_t)G::LDS_BYTES + 64 * 8 + (size_t)p.K * 8;
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)gemm_kernel<64, 64, A_ROWK_LN, B_ROWK, 2, BK>,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);
  if (attr_ok != hipSuccess) return attr_ok;
  if (lds > 156 * 1024) return hipErrorInvalidValue;
  dim3 grid((p.M + 63) / 64, (p.N + 63) / 64, p.split_k);
  hipLaunchKernelGGL((gemm_kernel<64, 64, A_ROWK_LN, B_ROWK, 2, BK>), grid, dim3(256), lds, s, p, aux);
  return hipGetLastError();
}

// halo tiles: ids 16.. (tile_halo_bm / tile_halo_bn), 3-deep B ring, window + ring in dynamic LDS
constexpr int HALO_NS = 3;
constexpr int HALO_LDS_MAX = 156 * 1024;  // 160 KiB less the paired kernel's static finalize scratch
__host__ __device__ constexpr int halo_bm(int t) {
  return t == 16 ? 64 : t == 17 ? 128 : t == 18 ? 128 : t == 19 ? 256 : t == 20 ? 128 : t == 21 ? 256 : t == 22 ? 64 : 64;
}
__host__ __device__ constexpr int halo_bn(int t) {
  return t == 16 ? 64 : t == 17 ? 64 : t == 18 ? 128 : t == 19 ? 32 : t == 20 ? 32 : t == 21 ? 64 : t == 22 ? 128 : 32;
}
inline size_t halo_lds_bytes(const HaloGeom& h, int bm, int bn) {
  const size_t win = (size_t)h.chunks * 16 + (size_t)HALO_NS * bn * BK * 2;
  const size_t epi = (size_t)bm * (bn + 4) * 4;
  return win > epi ? win : epi;
}

template <int BM, int BN, int BMD>
hipError_t launch_halo_t(const EncdiffGemmArgs& p, const GemmAux& aux, hipStream_t s) {
  static const hipError_t attr_ok = hipFuncSetAttribute(
      (const void*)gemm_kernel<BM, BN, A_HALO, BMD, HALO_NS, BK>, hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
  if (attr_ok != hipSuccess) return attr_ok;
  dim3 grid(p.M / BM, (p.N + BN - 1) / BN, p.split_k);
  hipLaunchKernelGGL((gemm_kernel<BM, BN, A_HALO, BMD, HALO_NS, BK>), grid, dim3(256), halo_lds_bytes(aux.halo, BM, BN), s,
                     p, aux);
  return hipGetLastError();
}

template <int BMD>
hipError_t launch_halo(const EncdiffGemmArgs& p, const GemmAux& aux, int tile, hipStream_t s) {
  switch (tile) {
    case 16: return launch_halo_t<64, 64, BMD>(p, aux, s);
    case 17: return launch_halo_t<128, 64, BMD>(p, aux, s);
    case 18: return launch_halo_t<128, 128, BMD>(p, aux, s);
    case 19: return launch_halo_t<256, 32, BMD>(p, aux, s);
    case 20: return launch_halo_t<128, 32, BMD>(p, aux, s);
    case 21: return launch_halo_t<256, 64, BMD>(p, aux, s);
    case 22: return launch_halo_t<64, 128, BMD>(p, aux, s);
    default: return launch_halo_t<64, 32, BMD>(p, aux, s);
  }
}

template <int AM, int BMD>
hipError_t launch_modes(const EncdiffGemmArgs& p, const GemmAux& aux, int tile, hipStream_t s) {
  if constexpr (AM == A_IM2COL && (BMD == B_ROWK || BMD == B_CONVD)) {
    if (tile >= 16) return launch_halo<BMD>(p, aux, tile, s);
  }
  switch (tile) {
    case 1: return launch_t<128, 128, AM, BMD>(p, aux, s);
    case 2: return launch_t<128, 64, AM, BMD>(p, aux, s);
    case 3: return launch_t<64, 128, AM, BMD>(p, aux, s);
    case 5: return launch_t<64, 64, AM, BMD, 4>(p, aux, s);
    case 6: return launch_t<64, 128, AM, BMD, 3>(p, aux, s);
    case 7: return launch_t<64, 64, AM, BMD, 2, 128>(p, aux, s);
    case 8: return launch_t<64, 128, AM, BMD, 2, 128>(p, aux, s);
    case 9: return launch_t<64, 64, AM, BMD, 6>(p, aux, s);
    case 10: return launch_t<64, 64, AM, BMD, 8>(p, aux, s);
    default: return launch_t<64, 64, AM, BMD>(p, aux, s);
  }
}

FDiv make_fdiv(int d) {
  FDiv f;
  f.d = d > 0 ? (uint32_t)d : 1u;
  f.mul = (1ull << 40) / f.d + 1;
  f.pad_ = 0;
  return f;
}

int pick_tile(const EncdiffGemmArgs& p) {
  int bm = (p.M <= 64) ? 64 : 128;
  int bn = (p.N <= 64) ? 64 : 128;
  auto blocks = [&](int a, int b) { return ((p.M + a - 1) / a) * ((p.N + b - 1) / b) * p.split_k; };
  if (blocks(bm, bn) < 512 && bm == 128) bm = 64;
  if (blocks(bm, bn) < 512 && bn == 128) bn = 64;
  if (bm == 128 && bn == 128) return 1;
  if (bm == 128) return 2;
  if (bn == 128) return 3;
  return 4;
}

int gcd_i(int a, int b) { return b ? gcd_i(b, a % b) : a; }

// Halo-tile eligibility and geometry (tiles 16..23): implicit-im2col A of a 3x3 (pad 1, optional
// nearest-up), VQ stride-2 or Encoder4 k4 s2 conv forward, or a plain 3x3 input gradient;
// BM pixels = whole rows of one image or whole images; window + B ring within 160 KiB of LDS.
int prepare_halo(const EncdiffGemmArgs& p, int tile, HaloGeom& h) {
  if (tile > 23 || p.a_mode != ENCDIFF_OPA_IM2COL) return ENCDIFF_ERR_UNSUPPORTED;
  const int rs = p.conv.resample;
  if (p.b_mode == ENCDIFF_OPB_ROWK) {
    if (rs != ENCDIFF_RESAMPLE_NONE && rs != ENCDIFF_RESAMPLE_UP2 && rs != ENCDIFF_RESAMPLE_STRIDE2 &&
        rs != ENCDIFF_RESAMPLE_K4S2)
      return ENCDIFF_ERR_UNSUPPORTED;
  } else if (p.b_mode != ENCDIFF_OPB_CONV_DGRAD || rs != ENCDIFF_RESAMPLE_NONE) {
    return ENCDIFF_ERR_UNSUPPORTED;
  }
  if (p.c_mode == ENCDIFF_OUT_F32_ATOMIC || p.c_mode == ENCDIFF_OUT_F32_ATOMIC_CONVW) return ENCDIFF_ERR_UNSUPPORTED;
  // split-K: each split stages and contracts its own slice of the source channels (gemm_tile)
  if (p.split_k > 1 && (p.conv.cin % (64 * p.split_k) || p.K % 64)) return ENCDIFF_ERR_SHAPE;
  const int bm = halo_bm(tile), bn = halo_bn(tile);
  const int H = p.conv.h, W = p.conv.w, HW = H * W, cin = p.conv.cin;
  if ((long)p.M != (long)p.conv.batch * HW || p.M % bm || bm % W || (HW % bm && bm % HW)) return ENCDIFF_ERR_SHAPE;
  const bool up = rs == ENCDIFF_RESAMPLE_UP2, s2 = rs == ENCDIFF_RESAMPLE_STRIDE2, k4 = rs == ENCDIFF_RESAMPLE_K4S2;
  if (up && ((H | W) & 1)) return ENCDIFF_ERR_SHAPE;
  h.s = (s2 || k4) ? 2 : 1;
  h.off = s2 ? 0 : -1;
  h.kt = k4 ? 4 : 3;
  if (p.K != h.kt * h.kt * cin || cin % 8) return ENCDIFF_ERR_SHAPE;
  h.lh = h.s * H;
  h.lw = h.s * W;
  h.ush = up ? 1 : 0;
  h.hs = up ? H / 2 : h.lh;
  h.ws = up ? W / 2 : h.lw;
  const int rows = bm / W < H ? bm / W : H;
  h.ni = bm > HW ? bm / HW : 1;
  h.hr = h.s * (rows - 1) + h.kt;
  h.hc = h.s * (W - 1) + h.kt;
  h.ch = cin / 8 / p.split_k;  // the split's channel slice
  h.npix = h.ni * h.hr * h.hc;
  h.chunks = (h.npix * h.ch + 255) & ~255;
  // bank swizzle: consecutive pixels advance q 16-B slots in the 16-slot bank row; g pixels share a
  // slot position, spread them over min(g, largest power of two dividing ch) slots
  const int q = h.ch % 16, g = q ? gcd_i(q, 16) : 16;
  int pw = 1;
  while (pw < 16 && h.ch % (2 * pw) == 0) pw *= 2;
  h.xmsk = (pw < g ? pw : g) - 1;
  int xsh = 0;
  while ((1 << xsh) < 16 / g) ++xsh;
  h.xsh = xsh;
  h.fch = make_fdiv(h.ch);
  h.fimg = make_fdiv(h.hr * h.hc);
  h.fhc = make_fdiv(h.hc);
  if (halo_lds_bytes(h, bm, bn) > (size_t)HALO_LDS_MAX) return ENCDIFF_ERR_SHAPE;
  return ENCDIFF_OK;
}

// Validated launch plan of one GEMM: the arguments the tile kernel sees (split-K slabs
// redirected into the workspace), the user's arguments for the finalize pass, aux constants.
struct GemmPlan {
  EncdiffGemmArgs p, user;
  GemmAux aux;
  int tile;
  bool ws_path;
  bool fold;  // split-K slabs combined in the kernel (no finalize pass)
};

// XCD-aware tile order (xcd_remap) per problem.  Measured per call over the step's GEMMs
// (tools/gemm_calls_time.py, round 4): it pays for the weight gradients whose A operand is
// k-outer (dY^T, deep split-K over pixels: the x / dY k-slices of 8 split-K parts and 8 M tiles
// stay in one L2; the 512x64x32768 linear pairs 22.4 -> 16.9 us) and LOSES for the forward /
// input-gradient convs (M = 2048 split-4 3x3 convs 14.6 -> 21.7 us: one XCD's 64 workgroups then
// start on the same two weight tiles at once).  ENCDIFF_GEMM_XCD: 0 off, 1 every GEMM, 2 (default)
// the k-outer-A GEMMs only.
int gemm_xcd_order(const EncdiffGemmArgs& p) {
  static const int v = [] {
    const char* e = getenv("ENCDIFF_GEMM_XCD");
    return e ? atoi(e) : 2;
  }();
  return v == 1 || (v == 2 && p.a_mode == ENCDIFF_OPA_ROWM);
}

int prepare(const EncdiffGemmArgs* pa, GemmPlan& g) {
  if (!pa || pa->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_ARG;  // fp32: encdiff_gemm only
  EncdiffGemmArgs p = *pa;
  if (p.M <= 0 || p.N <= 0 || p.K <= 0) return ENCDIFF_ERR_SHAPE;
  if (p.split_k < 1) p.split_k = 1;
  const bool ws_path = p.split_k > 1 && (p.c_mode == ENCDIFF_OUT_BF16 || p.c_mode == ENCDIFF_OUT_F32 ||
                                         p.c_mode == ENCDIFF_OUT_F32_ACCUM);
  if (ws_path && !p.workspace) return ENCDIFF_ERR_ARG;
  const bool k_inner = p.a_mode != ENCDIFF_OPA_ROWM || p.b_mode == ENCDIFF_OPB_ROWK;
  if (k_inner && p.K % 8) return ENCDIFF_ERR_SHAPE;
  if (p.a_mode == ENCDIFF_OPA_ROWM && p.M % 8) return ENCDIFF_ERR_SHAPE;
  if (p.b_mode != ENCDIFF_OPB_ROWK && p.N % 8) return ENCDIFF_ERR_SHAPE;
  const bool im2col = p.a_mode == ENCDIFF_OPA_IM2COL || p.b_mode == ENCDIFF_OPB_IM2COL;
  if (im2col && (p.conv.cin % 8)) return ENCDIFF_ERR_SHAPE;
  // exact fdiv range (pixel indices < 2^24, divisors < 2^16) and single-load im2col modes
  if (im2col && ((long)p.conv.batch * p.conv.h * p.conv.w >= (1L << 24) || p.conv.h * p.conv.w >= (1 << 16)))
    return ENCDIFF_ERR_SHAPE;
  if (im2col && p.conv.resample == ENCDIFF_RESAMPLE_DOWN2) return ENCDIFF_ERR_UNSUPPORTED;
  if (im2col && p.conv.resample == ENCDIFF_RESAMPLE_K4S2_TP) {  // parity-major rows, one parity per tile
    if (p.a_mode != ENCDIFF_OPA_IM2COL || p.b_mode != ENCDIFF_OPB_CONV_DGRAD) return ENCDIFF_ERR_UNSUPPORTED;
    if ((p.conv.h | p.conv.w) & 1 || (long)p.M != (long)p.conv.batch * p.conv.h * p.conv.w ||
        (p.M >> 2) % 128 || p.K != 4 * p.conv.cin)
      return ENCDIFF_ERR_SHAPE;
    if (p.c_mode == ENCDIFF_OUT_F32_ATOMIC || p.c_mode == ENCDIFF_OUT_F32_ATOMIC_CONVW) return ENCDIFF_ERR_UNSUPPORTED;
  }
  if (p.K >= (1 << 24)) return ENCDIFF_ERR_SHAPE;
  {  // the staging loads address every operand by 32-bit byte offsets from its base
    const long src = (long)p.conv.batch * p.conv.h * p.conv.w * 4 * p.conv.ld_src * 2;  // im2col source
    long ea = 0, eb = 0;
    if (p.a_mode == ENCDIFF_OPA_ROWK) ea = ((long)(p.M - 1) * p.lda + p.K) * 2;
    else if (p.a_mode == ENCDIFF_OPA_ROWM) ea = ((long)(p.K - 1) * p.lda + p.M) * 2;
    else ea = src;
    if (p.b_mode == ENCDIFF_OPB_ROWK) eb = ((long)(p.N - 1) * p.ldb + p.K) * 2;
    else if (p.b_mode == ENCDIFF_OPB_ROWN) eb = ((long)(p.K - 1) * p.ldb + p.N) * 2;
    else if (p.b_mode == ENCDIFF_OPB_CONV_DGRAD) eb = ((long)p.conv_cout * p.ldb + 16L * p.N) * 2;
    else eb = src;
    if (ea >= 0x7FFFFFF0L || eb >= 0x7FFFFFF0L) return ENCDIFF_ERR_SHAPE;
  }
  if (p.bias_grad && p.a_mode != ENCDIFF_OPA_ROWM) return ENCDIFF_ERR_ARG;
  if (p.gn_stats && (p.c_mode != ENCDIFF_OUT_BF16 || p.split_k != 1 || p.M % 64 || p.ld_gn_stats < p.N))
    return ENCDIFF_ERR_ARG;
  if (p.ln_y) {  // the tile must span every column: N <= BN, 8-column vectors
    const int bn = (p.tile == 1 || p.tile == 3 || p.tile == 6 || p.tile == 8) ? 128 : 64;
    if (p.c_mode != ENCDIFF_OUT_BF16 || p.split_k != 1 || !p.tile || p.N > bn || p.N % 8 || p.ld_ln_y % 8 ||
        !p.ln_gamma || !p.ln_beta || !p.ln_stats)
      return ENCDIFF_ERR_ARG;
  }
  if (p.c_mode == ENCDIFF_OUT_BF16_GEGLU || p.c_mode == ENCDIFF_OUT_BF16_GEGLU_BWD) {
    const bool fwd = p.c_mode == ENCDIFF_OUT_BF16_GEGLU;
    if (!p.aux || p.resid || p.split_k != 1 || p.N % 8 || p.ldc % 8 || p.ld_aux % 8) return ENCDIFF_ERR_ARG;
    if (fwd && (p.a_mode != ENCDIFF_OPA_ROWK || p.b_mode != ENCDIFF_OPB_ROWK || p.N % 128)) return ENCDIFF_ERR_ARG;
  }
  if (p.agn_gamma) {  // GroupNorm in the A staging: forward 3x3 conv, 64x64 tiles
    if (p.a_mode != ENCDIFF_OPA_IM2COL || p.b_mode != ENCDIFF_OPB_ROWK || p.c_mode != ENCDIFF_OUT_BF16 ||
        !p.agn_beta || p.ln_y)
      return ENCDIFF_ERR_ARG;
    if (p.conv.resample != ENCDIFF_RESAMPLE_NONE && p.conv.resample != ENCDIFF_RESAMPLE_UP2)
      return ENCDIFF_ERR_UNSUPPORTED;
    if (p.conv.cin % 32 || p.conv.cin > 1024 || p.K != 9 * p.conv.cin ||
        (long)p.M != (long)p.conv.batch * p.conv.h * p.conv.w)
      return ENCDIFF_ERR_SHAPE;
    if (p.tile != 0 && p.tile != 4) return ENCDIFF_ERR_UNSUPPORTED;
    p.tile = 4;
  }
  if (p.lna_gamma) {  // LayerNorm in the A staging: linear forward, 64x64 tiles, no split
    if (p.a_mode != ENCDIFF_OPA_ROWK || p.b_mode != ENCDIFF_OPB_ROWK || p.c_mode != ENCDIFF_OUT_BF16 ||
        !p.lna_beta || p.ln_y || p.agn_gamma || p.split_k != 1)
      return ENCDIFF_ERR_ARG;
    if (p.K % 8 || p.K > 1024 || p.lda % 8 || ((uintptr_t)p.a & 15)) return ENCDIFF_ERR_SHAPE;
    if (p.tile != 0 && p.tile != 4) return ENCDIFF_ERR_UNSUPPORTED;
    p.tile = 4;
  }
  g.tile = p.tile ? p.tile : pick_tile(p);
  g.aux.halo = HaloGeom{};
  if (g.tile >= 32 && g.tile <= 34) {  // 3x3 conv weight gradient kernel (WG3)
    const int rc = wg3_check(p);
    if (rc != ENCDIFF_OK) return rc;
  } else if (g.tile == 36) {  // linear weight gradient kernel (WGL)
    const int rc = wgl_check(p);
    if (rc != ENCDIFF_OK) return rc;
  } else if (g.tile >= 16) {
    const int rc = prepare_halo(p, g.tile, g.aux.halo);
    if (rc != ENCDIFF_OK) return rc;
  }
  g.user = p;
  g.ws_path = ws_path;
  if (ws_path) {  // per-split fp32 slabs (plain stores); epilogue in the finalize pass
    p.c = p.workspace; p.ldc = p.N; p.c_mode = ENCDIFF_OUT_F32; p.alpha = 1.f;
    p.bias = nullptr; p.resid = nullptr;
  }
  // in-kernel split-K combine: vectorised slab / output rows, plain row mapping, no bias gradient
  g.aux.fold = SplitFold{};
  g.fold = false;
  if (ws_path && p.split_counters && p.a_mode != ENCDIFF_OPA_ROWM && !p.bias_grad && p.N % 8 == 0 &&
      !(im2col && p.conv.resample == ENCDIFF_RESAMPLE_K4S2_TP) && g.user.ldc % 8 == 0 &&
      ((uintptr_t)g.user.c & 15) == 0 && ((uintptr_t)p.workspace & 15) == 0 &&
      (!g.user.bias || ((uintptr_t)g.user.bias & 15) == 0) &&
      (!g.user.resid || (g.user.ld_resid % 8 == 0 && ((uintptr_t)g.user.resid & 15) == 0))) {
    g.fold = true;
    g.aux.fold = SplitFold{p.split_counters, g.user.c, g.user.ldc, g.user.c_mode, g.user.alpha, g.user.bias,
                           (const bf16_t*)g.user.resid, g.user.ld_resid};
  }
  g.p = p;
  g.aux.xcd = gemm_xcd_order(p);
  g.aux.cin = make_fdiv(p.conv.cin);
  g.aux.cout = make_fdiv(p.conv_cout);
  const bool tp = im2col && p.conv.resample == ENCDIFF_RESAMPLE_K4S2_TP;
  g.aux.hw = make_fdiv(tp ? (p.conv.h >> 1) * (p.conv.w >> 1) : p.conv.h * p.conv.w);  // output grid
  g.aux.w = make_fdiv(tp ? p.conv.w >> 1 : p.conv.w);
  return ENCDIFF_OK;
}

int fin_blocks(const EncdiffGemmArgs& u) {
  const long total = (long)u.M * u.N;
  const long per = fin_per_block(u);
  long g = (total + per - 1) / per;
  if (u.bias_grad && (u.M + 63) / 64 > g) g = (u.M + 63) / 64;
  return (int)(g > 2048 ? 2048 : g);
}

int launch_one(const GemmPlan& g, hipStream_t s) {
  const int am = g.p.a_mode, bm = g.p.b_mode;
  hipError_t e;
  if (g.tile >= 32 && g.tile <= 34) e = wg3_launch(g.p, g.tile, g.user, 0, s);
  else if (g.tile == 36) e = wgl_launch(g.p, g.user, 0, s);
  else if (am == ENCDIFF_OPA_ROWK && bm == ENCDIFF_OPB_ROWK)
    e = g.p.lna_gamma ? launch_lna(g.p, g.aux, s) : launch_modes<A_ROWK, B_ROWK>(g.p, g.aux, g.tile, s);
  else if (am == ENCDIFF_OPA_IM2COL && bm == ENCDIFF_OPB_ROWK)
    e = g.p.agn_gamma ? launch_agn(g.p, g.aux, s) : launch_modes<A_IM2COL, B_ROWK>(g.p, g.aux, g.tile, s);
  else if (am == ENCDIFF_OPA_ROWK && bm == ENCDIFF_OPB_ROWN) e = launch_modes<A_ROWK, B_ROWN>(g.p, g.aux, g.tile, s);
  else if (am == ENCDIFF_OPA_IM2COL && bm == ENCDIFF_OPB_CONV_DGRAD)
    e = launch_modes<A_IM2COL, B_CONVD>(g.p, g.aux, g.tile, s);
  else if (am == ENCDIFF_OPA_ROWM && bm == ENCDIFF_OPB_ROWN) e = launch_modes<A_ROWM, B_ROWN>(g.p, g.aux, g.tile, s);
  else if (am == ENCDIFF_OPA_ROWM && bm == ENCDIFF_OPB_IM2COL) e = launch_modes<A_ROWM, B_IM2COL>(g.p, g.aux, g.tile, s);
  else return ENCDIFF_ERR_UNSUPPORTED;
  if (e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
  if (g.ws_path && !g.fold) {
    hipLaunchKernelGGL(gemm_finalize_kernel, dim3((unsigned)fin_blocks(g.user)), dim3(256), 0, s, g.user);
    e = hipGetLastError();
    if (e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
  }
  return ENCDIFF_OK;
}

template <int AM1, int BMD1, int BM2, int BN2, int AM2, int BMD2, int NS2 = 2, int KB2 = BK, int KB1 = BK, int NS1 = 2>
hipError_t launch_pair_t(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  using G1 = Gemm<64, 64, AM1, BMD1, NS1, KB1>;
  using G2 = Gemm<BM2, BN2, AM2, BMD2, NS2, KB2>;
  constexpr size_t lds = G1::LDS_BYTES > G2::LDS_BYTES ? G1::LDS_BYTES : G2::LDS_BYTES;
  static const hipError_t attr_ok = hipFuncSetAttribute(
      (const void*)gemm2_kernel<AM1, BMD1, BM2, BN2, AM2, BMD2, NS2, KB2, KB1, NS1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr_ok != hipSuccess) return attr_ok;
  const int gx1 = (g1.p.M + 63) / 64, gy1 = (g1.p.N + 63) / 64;
  const int gx2 = (g2.p.M + BM2 - 1) / BM2, gy2 = (g2.p.N + BN2 - 1) / BN2;
  const long nb = (long)gx1 * gy1 * g1.p.split_k + (long)gx2 * gy2 * g2.p.split_k + nf;
  hipLaunchKernelGGL((gemm2_kernel<AM1, BMD1, BM2, BN2, AM2, BMD2, NS2, KB2, KB1, NS1>), dim3((unsigned)nb), dim3(256), lds, s, g1.p,
                     g1.aux, g2.p, g2.aux, gx1, gy1, gx2, gy2, pf, nf);
  return hipGetLastError();
}

// paired launch whose input gradient runs on a halo tile: dynamic LDS = the larger of the two
template <int AM1, int BMD1, int BM2, int BN2, int KB1>
hipError_t launch_pair_halo_t(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  using G1 = Gemm<64, 64, AM1, BMD1, 2, KB1>;
  auto kern = gemm2_kernel<AM1, BMD1, BM2, BN2, A_HALO, B_CONVD, HALO_NS, BK, KB1>;
  static const hipError_t attr_ok =
      hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
  if (attr_ok != hipSuccess) return attr_ok;
  size_t lds = halo_lds_bytes(g2.aux.halo, BM2, BN2);
  if ((size_t)G1::LDS_BYTES > lds) lds = G1::LDS_BYTES;
  const int gx1 = (g1.p.M + 63) / 64, gy1 = (g1.p.N + 63) / 64;
  const int gx2 = g2.p.M / BM2, gy2 = (g2.p.N + BN2 - 1) / BN2;
  const long nb = (long)gx1 * gy1 * g1.p.split_k + (long)gx2 * gy2 * g2.p.split_k + nf;
  hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(256), lds, s, g1.p, g1.aux, g2.p, g2.aux, gx1, gy1, gx2, gy2, pf, nf);
  return hipGetLastError();
}

template <int AM1, int BMD1, int KB1>
hipError_t launch_pair_halo(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  switch (g2.tile) {
    case 16: return launch_pair_halo_t<AM1, BMD1, 64, 64, KB1>(g1, g2, pf, nf, s);
    case 17: return launch_pair_halo_t<AM1, BMD1, 128, 64, KB1>(g1, g2, pf, nf, s);
    case 18: return launch_pair_halo_t<AM1, BMD1, 128, 128, KB1>(g1, g2, pf, nf, s);
    case 22: return launch_pair_halo_t<AM1, BMD1, 64, 128, KB1>(g1, g2, pf, nf, s);
    default: return hipErrorInvalidValue;
  }
}

template <int AM1, int BMD1, int AM2, int BMD2>
hipError_t launch_pair_tiles(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf,
                             hipStream_t s) {
  if constexpr (AM2 == A_IM2COL && BMD2 == B_CONVD) {
    if (g2.tile >= 16) {
      return g1.tile == 7 ? launch_pair_halo<AM1, BMD1, 128>(g1, g2, pf, nf, s)
                          : launch_pair_halo<AM1, BMD1, BK>(g1, g2, pf, nf, s);
    }
  }
  if (g1.tile == 5) {  // weight gradient with a 4-deep ring (64 KB of LDS): every k-tile of a short split in flight
    return launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 2, 64, 64, 4>(g1, g2, pf, nf, s);
  }
  if (g1.tile == 9 || g1.tile == 10) {  // 6- / 8-deep rings (96 / 128 KB): one workgroup per CU, all loads in flight
    const bool d6 = g1.tile == 9;
    switch (g2.tile) {
      case 9: return d6 ? launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 6, 64, 64, 6>(g1, g2, pf, nf, s)
                        : launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 6, 64, 64, 8>(g1, g2, pf, nf, s);
      case 10: return d6 ? launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 8, 64, 64, 6>(g1, g2, pf, nf, s)
                         : launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 8, 64, 64, 8>(g1, g2, pf, nf, s);
      default: return d6 ? launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 2, 64, 64, 6>(g1, g2, pf, nf, s)
                         : launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 2, 64, 64, 8>(g1, g2, pf, nf, s);
    }
  }
  if (g1.tile == 7) {  // weight gradient with 128-deep k stages (64 KB of LDS): dgrad tile 7 or 64x64
    if (g2.tile == 7) return launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 2, 128, 128>(g1, g2, pf, nf, s);
    return launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 2, 64, 128>(g1, g2, pf, nf, s);
  }
  switch (g2.tile) {
    case 1: return launch_pair_t<AM1, BMD1, 128, 128, AM2, BMD2>(g1, g2, pf, nf, s);
    case 2: return launch_pair_t<AM1, BMD1, 128, 64, AM2, BMD2>(g1, g2, pf, nf, s);
    case 3: return launch_pair_t<AM1, BMD1, 64, 128, AM2, BMD2>(g1, g2, pf, nf, s);
    case 5: return launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 4>(g1, g2, pf, nf, s);
    case 6: return launch_pair_t<AM1, BMD1, 64, 128, AM2, BMD2, 3>(g1, g2, pf, nf, s);
    case 7: return launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2, 2, 128>(g1, g2, pf, nf, s);
    case 8: return launch_pair_t<AM1, BMD1, 64, 128, AM2, BMD2, 2, 128>(g1, g2, pf, nf, s);
    default: return launch_pair_t<AM1, BMD1, 64, 64, AM2, BMD2>(g1, g2, pf, nf, s);
  }
}

template <int W, bool UP, int BM2, int BN2, int AM2, int BMD2, int NS2>
hipError_t wg3pair_launch_t(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  static const hipError_t attr_ok =
      hipFuncSetAttribute((const void*)wgrad3x3_kernel<W, UP, WG3_PAIR_NS, 4, BM2, BN2, AM2, BMD2, NS2>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, HALO_LDS_MAX);
  if (attr_ok != hipSuccess) return attr_ok;
  size_t lds = wg3_lds<W, WG3_PAIR_NS, 4>();
  if constexpr (AM2 == A_HALO) {
    const size_t h = halo_lds_bytes(g2.aux.halo, BM2, BN2);
    if (h > lds) lds = h;
  } else {
    constexpr size_t l2 = Gemm<BM2, BN2, AM2, BMD2, NS2, BK>::LDS_BYTES;
    if (l2 > lds) lds = l2;
  }
  const int n1 = (g1.p.M / 32) * (g1.p.conv.cin / 16) * g1.p.split_k;
  const int gx2 = AM2 == A_HALO ? g2.p.M / BM2 : (g2.p.M + BM2 - 1) / BM2, gy2 = (g2.p.N + BN2 - 1) / BN2;
  const long nb = (long)n1 + (long)gx2 * gy2 * g2.p.split_k + nf;
  hipLaunchKernelGGL((wgrad3x3_kernel<W, UP, WG3_PAIR_NS, 4, BM2, BN2, AM2, BMD2, NS2>), dim3((unsigned)nb), dim3(256), lds, s,
                     g1.p, n1, pf, nf, g2.p, g2.aux, gx2, gy2);
  return hipGetLastError();
}

template <int W, bool UP>
hipError_t wg3pair_launch_w(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  switch (g2.tile) {
    case 4: return wg3pair_launch_t<W, UP, 64, 64, A_IM2COL, B_CONVD, 2>(g1, g2, pf, nf, s);
    case 2: return wg3pair_launch_t<W, UP, 128, 64, A_IM2COL, B_CONVD, 2>(g1, g2, pf, nf, s);
    case 16: return wg3pair_launch_t<W, UP, 64, 64, A_HALO, B_CONVD, HALO_NS>(g1, g2, pf, nf, s);
    case 17: return wg3pair_launch_t<W, UP, 128, 64, A_HALO, B_CONVD, HALO_NS>(g1, g2, pf, nf, s);
    case 22: return wg3pair_launch_t<W, UP, 64, 128, A_HALO, B_CONVD, HALO_NS>(g1, g2, pf, nf, s);
    default: return hipErrorInvalidValue;
  }
}

// the input-gradient tiles the paired WG3 launch covers
bool wg3pair_ok(const GemmPlan& g1, const GemmPlan& g2) {
  return g1.tile == 32 && g2.p.a_mode == ENCDIFF_OPA_IM2COL && g2.p.b_mode == ENCDIFF_OPB_CONV_DGRAD &&
         (g2.tile == 4 || g2.tile == 2 || g2.tile == 16 || g2.tile == 17 || g2.tile == 22);
}

hipError_t wg3pair_launch(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  const bool up = g1.p.conv.resample == ENCDIFF_RESAMPLE_UP2;
  switch (g1.p.conv.w) {
    case 4: return up ? wg3pair_launch_w<4, true>(g1, g2, pf, nf, s) : wg3pair_launch_w<4, false>(g1, g2, pf, nf, s);
    case 8: return up ? wg3pair_launch_w<8, true>(g1, g2, pf, nf, s) : wg3pair_launch_w<8, false>(g1, g2, pf, nf, s);
    default: return up ? wg3pair_launch_w<16, true>(g1, g2, pf, nf, s) : wg3pair_launch_w<16, false>(g1, g2, pf, nf, s);
  }
}

template <int BM2, int BN2, int NS2, int KB2>
hipError_t wglpair_launch_t(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  using G2 = Gemm<BM2, BN2, A_ROWK, B_ROWN, NS2, KB2>;
  constexpr size_t l1 = wgl_lds<WGL_PAIR_NS>(), lds = l1 > G2::LDS_BYTES ? l1 : G2::LDS_BYTES;
  static const hipError_t attr_ok =
      hipFuncSetAttribute((const void*)wgradlin_kernel<WGL_PAIR_NS, BM2, BN2, A_ROWK, B_ROWN, NS2, KB2>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (attr_ok != hipSuccess) return attr_ok;
  const int n1 = (g1.p.M / 64) * (g1.p.N / 64) * g1.p.split_k;
  const int gx2 = (g2.p.M + BM2 - 1) / BM2, gy2 = (g2.p.N + BN2 - 1) / BN2;
  const long nb = (long)n1 + (long)gx2 * gy2 * g2.p.split_k + nf;
  hipLaunchKernelGGL((wgradlin_kernel<WGL_PAIR_NS, BM2, BN2, A_ROWK, B_ROWN, NS2, KB2>), dim3((unsigned)nb), dim3(256), lds,
                     s, g1.p, n1, pf, nf, g2.p, g2.aux, gx2, gy2);
  return hipGetLastError();
}

bool wglpair_ok(const GemmPlan& g1, const GemmPlan& g2) {
  return g1.tile == 36 && g2.p.a_mode == ENCDIFF_OPA_ROWK && g2.p.b_mode == ENCDIFF_OPB_ROWN && !g2.fold &&
         (g2.tile >= 1 && g2.tile <= 5 || g2.tile == 7);
}

hipError_t wglpair_launch(const GemmPlan& g1, const GemmPlan& g2, const EncdiffGemmArgs& pf, int nf, hipStream_t s) {
  switch (g2.tile) {
    case 1: return wglpair_launch_t<128, 128, 2, BK>(g1, g2, pf, nf, s);
    case 2: return wglpair_launch_t<128, 64, 2, BK>(g1, g2, pf, nf, s);
    case 3: return wglpair_launch_t<64, 128, 2, BK>(g1, g2, pf, nf, s);
    case 5: return wglpair_launch_t<64, 64, 4, BK>(g1, g2, pf, nf, s);
    case 7: return wglpair_launch_t<64, 64, 2, 128>(g1, g2, pf, nf, s);
    default: return wglpair_launch_t<64, 64, 2, BK>(g1, g2, pf, nf, s);
  }
}

hipError_t launch_finalize(const EncdiffGemmArgs& u, hipStream_t s) {
  hipLaunchKernelGGL(gemm_finalize_kernel, dim3((unsigned)fin_blocks(u)), dim3(256), 0, s, u);
  return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Grouped weight gradients (encdiff_wgrad_group_plan / _launch): the weight gradients of a whole
// backward region -- every nn.Linear / 3x3 conv / skip conv of the output blocks, or of the rest
// of the UNet (openaimodel_enc.py:255-275, attention.py:159-167, 211-261) -- in ONE grid, after
// the region's input-gradient chain has produced every dY.  Alone, each of these problems (output
// a few KB, K = 2 048 .. 32 768 pixels) fills the chip only through split-K, whose fp32 slabs and
// finalize passes were half the GEMM family's excess traffic; together there are thousands of
// output parts, so every problem runs WHOLE (split_k 1): each output element is produced by one
// workgroup in one ordered sum (reproducible), no slabs, no finalize.  The workgroup bodies are
// the WG3 (3x3 conv, h in {4, 8, 16}) and WGL (linear, 64 x 64 parts) kernels' and the generic
// 64 x 64 tile for the rest (2x2 convs, narrow / short-K linears).  Work items are ordered by
// cost, longest first, so the list scheduling of the dispatcher balances the CUs.
struct WgProb {
  EncdiffGemmArgs p;
  GemmAux aux;
  int kind, gx, nblk, pad_;
};
struct WgBlobHead {
  int magic, n_probs, n_items, lds;
  long probs_off, items_off, bytes, pad_;
};
constexpr int WGG_MAGIC = 0x57474731;  // "WGG1"
constexpr int WGG_WG3_NS = 3, WGG_WGL_NS = 2;
// kinds: 0..5 WG3 (w 16 / 8 / 4) x (resample none / up2), 6 WGL, 7 generic linear, 8 generic conv
enum { WGK_WGL = 6, WGK_GEN_LIN = 7, WGK_GEN_CONV = 8 };
constexpr size_t cmax(size_t a, size_t b) { return a > b ? a : b; }
constexpr size_t WGG_LDS =
    cmax(cmax(cmax(wg3_lds<16, WGG_WG3_NS, 4>(), wg3_lds<8, WGG_WG3_NS, 4>()), cmax(wg3_lds<4, WGG_WG3_NS, 4>(),
         wgl_lds<WGG_WGL_NS>())), cmax((size_t)Gemm<64, 64, A_ROWM, B_ROWN, 2, BK>::LDS_BYTES,
                                       (size_t)Gemm<64, 64, A_ROWM, B_IM2COL, 2, BK>::LDS_BYTES));

__global__ __launch_bounds__(256) void wgrad_group_kernel(const WgProb* __restrict__ probs,
                                                          const int* __restrict__ items) {
  extern __shared__ __attribute__((aligned(16))) char wsm[];
  const int it = items[blockIdx.x];
  if (it < 0) return;
  const int pi = it >> 20, loc = it & 0xFFFFF;
  const int kind = probs[pi].kind;
  const EncdiffGemmArgs p = probs[pi].p;  // read before any store: scalar loads
  const SplitFold fold = probs[pi].aux.fold;
  const SplitFold* fp = fold.cnt ? &fold : nullptr;  // chunks combined in the kernel
  switch (kind) {
    case 0: wgrad3x3_body<16, false, WGG_WG3_NS, 4, 9001>(p, loc, wsm, fp); return;
    case 1: wgrad3x3_body<16, true, WGG_WG3_NS, 4, 9002>(p, loc, wsm, fp); return;
    case 2: wgrad3x3_body<8, false, WGG_WG3_NS, 4, 9003>(p, loc, wsm, fp); return;
    case 3: wgrad3x3_body<8, true, WGG_WG3_NS, 4, 9004>(p, loc, wsm, fp); return;
    case 4: wgrad3x3_body<4, false, WGG_WG3_NS, 4, 9005>(p, loc, wsm, fp); return;
    case 5: wgrad3x3_body<4, true, WGG_WG3_NS, 4, 9006>(p, loc, wsm, fp); return;
    case WGK_WGL: wgradlin_body<WGG_WGL_NS, 9007>(p, loc, wsm, fp); return;
    default: {
      const GemmAux aux = probs[pi].aux;
      const int gx = probs[pi].gx;
      if (kind == WGK_GEN_LIN)
        gemm_tile<64, 64, A_ROWM, B_ROWN, 2, BK>(p, aux, loc % gx, loc / gx, 0, (bf16_t*)wsm);
      else
        gemm_tile<64, 64, A_ROWM, B_IM2COL, 2, BK>(p, aux, loc % gx, loc / gx, 0, (bf16_t*)wsm);
      return;
    }
  }
}

// Scratch the group's split-K chunks use: fp32 slabs (their own region of the caller's workspace)
// and one ticket per split output part (the caller's zeroed counter array; left zero).
struct WgScratch {
  float* ws;
  long ws_floats, ws_used;
  int* cnt;
  int n_cnt, cnt_used;
};

// 32-pixel / 32-token stages one wave of a group workgroup may run in sequence: deeper problems are
// cut into chunks of whole images / token ranges, combined in the kernel (wg_last_chunk).  At one
// or two waves per SIMD a wave's stage loop is latency-bound, so a long sequence would be the
// group's critical path (a whole 16x16 problem: 256 stages, ~120 us).  ENCDIFF_WGG_STAGES (32: a
// 16-stage plan of the WGL body at K = 8192 gave wrong sums in test_wgrad_group -- not pursued, the
// fused transformer backward uses its own kernel, encdiff_st_wgrad).
int wgg_stages() {
  static const int v = [] {
    const char* e = getenv("ENCDIFF_WGG_STAGES");
    return e ? atoi(e) : 32;
  }();
  return v;
}

// one problem of a group: the first body that accepts it (WG3, WGL, generic 64 x 64 tile), with
// the chunk count (split_k) that keeps each wave's stage sequence within wgg_stages()
int wg_prepare(const EncdiffGemmArgs& in, WgProb& w, double& block_flops, WgScratch& sc) {
  if (in.dtype != ENCDIFF_DT_BF16 || in.a_mode != ENCDIFF_OPA_ROWM) return ENCDIFF_ERR_ARG;
  if (in.c_mode != ENCDIFF_OUT_F32 && in.c_mode != ENCDIFF_OUT_F32_ACCUM) return ENCDIFF_ERR_UNSUPPORTED;
  if (in.b_mode != ENCDIFF_OPB_IM2COL && in.b_mode != ENCDIFF_OPB_ROWN) return ENCDIFF_ERR_UNSUPPORTED;
  EncdiffGemmArgs q = in;
  q.split_k = 1;
  q.workspace = nullptr;
  q.split_counters = nullptr;
  GemmPlan g;
  const bool conv = q.b_mode == ENCDIFF_OPB_IM2COL;
  q.tile = conv ? 32 : 36;
  if (prepare(&q, g) == ENCDIFF_OK) {
    int nparts, split = 1;
    if (conv) {
      const int wi = q.conv.w == 16 ? 0 : (q.conv.w == 8 ? 1 : 2);
      w.kind = 2 * wi + (q.conv.resample == ENCDIFF_RESAMPLE_UP2 ? 1 : 0);
      nparts = (q.M / 32) * (q.conv.cin / 16);
      const int ni = q.conv.w == 16 ? 1 : 2, rows = q.conv.w == 4 ? 4 : 2;
      auto spw = [&](int sp) {  // stages per wave, 0 when the chunking does not divide
        if (q.conv.batch % (sp * ni)) return 0;
        const int nst = (q.conv.batch / sp / ni) * (q.conv.h / rows);
        return nst % 4 ? 0 : nst / 4;
      };
      while (spw(split) > wgg_stages() && spw(2 * split) > 0) split *= 2;
      block_flops = 2.0 * 32 * 9 * 16 * (double)q.K / split;
    } else {
      w.kind = WGK_WGL;
      nparts = (q.M / 64) * (q.N / 64);
      while (q.K / (split * 128) > wgg_stages() && q.K % (2 * split * 128) == 0) split *= 2;
      block_flops = 2.0 * 64 * 64 * (double)q.K / split;
    }
    if (split > 1) {  // slabs + tickets, or whole when the scratch is exhausted
      // (regions 128-B aligned: a cache line never holds two problems' chunks -- see wg_last_chunk)
      const long need = ((long)split * q.M * q.N + (q.bias_grad ? (long)split * q.M : 0) + 31) & ~31L;
      if (sc.ws && sc.cnt && sc.ws_used + need <= sc.ws_floats && sc.cnt_used + nparts <= sc.n_cnt) {
        EncdiffGemmArgs qs = q;
        qs.split_k = split;
        qs.workspace = sc.ws + sc.ws_used;
        if (prepare(&qs, g) == ENCDIFF_OK) {
          g.aux.fold = SplitFold{sc.cnt + sc.cnt_used, g.user.c, g.user.ldc, g.user.c_mode, g.user.alpha,
                                 nullptr, nullptr, 0};
          sc.ws_used += need;
          sc.cnt_used += nparts;
        } else {
          split = 1;
        }
      } else {
        split = 1;
      }
      if (split == 1 && prepare(&q, g) != ENCDIFF_OK) return ENCDIFF_ERR_SHAPE;
    }
    if (split == 1) block_flops = (conv ? 2.0 * 32 * 9 * 16 : 2.0 * 64 * 64) * (double)q.K;
    w.nblk = nparts * split;
    w.gx = 0;
  } else {
    q.tile = 4;
    const int rc = prepare(&q, g);
    if (rc != ENCDIFF_OK) return rc;
    if (g.ws_path) return ENCDIFF_ERR_ARG;
    w.kind = conv ? WGK_GEN_CONV : WGK_GEN_LIN;
    w.gx = (q.M + 63) / 64;
    w.nblk = w.gx * ((q.N + 63) / 64);
    block_flops = 2.0 * 64 * 64 * (double)q.K;
  }
  w.p = g.p;
  w.aux = g.aux;
  w.aux.xcd = 0;
  w.pad_ = 0;
  return ENCDIFF_OK;
}

}  // namespace

// Work-item order of a group.  Blocks of one problem read the same dY / x rows (the whole K range:
// nothing is split), so they are kept on one XCD, whose L2 then serves the re-reads; problems go
// to the least-loaded XCD, largest first (those with more blocks than an XCD holds at once are
// cut into runs of consecutive blocks -- consecutive parts share their dY columns), and each XCD
// runs its blocks longest first.  Blocks are dealt round-robin over the XCDs by index (MI355X
// microarch guide: b and b + 8 share an XCD), so XCD x's list occupies indices x, x + 8, ...;
// shorter lists are padded with empty items.  ENCDIFF_WGG_ORDER=0: one global longest-first list.
static std::vector<int> wg_items(const std::vector<WgProb>& w, const std::vector<double>& cost) {
  const int n = (int)w.size();
  static const int order_mode = [] {
    const char* e = getenv("ENCDIFF_WGG_ORDER");
    return e ? atoi(e) : 1;
  }();
  std::vector<int> order((size_t)n);
  for (int i = 0; i < n; ++i) order[i] = i;
  std::vector<int> items;
  if (order_mode == 0) {
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    for (int i : order)
      for (int b = 0; b < w[i].nblk; ++b) items.push_back((i << 20) | b);
    return items;
  }
  constexpr int NX = 8, RUN = 64;  // XCDs; blocks of one problem per XCD run (32 CUs x 2 workgroups)
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return cost[a] * w[a].nblk > cost[b] * w[b].nblk; });
  std::vector<std::vector<int>> q(NX);
  double load[NX] = {0};
  for (int i : order) {
    for (int b0 = 0; b0 < w[i].nblk; b0 += RUN) {
      const int b1 = std::min(w[i].nblk, b0 + RUN);
      int x = 0;
      for (int k = 1; k < NX; ++k)
        if (load[k] < load[x]) x = k;
      load[x] += cost[i] * (b1 - b0);
      for (int b = b0; b < b1; ++b) q[x].push_back((i << 20) | b);
    }
  }
  size_t len = 0;
  for (auto& v : q) {
    std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return cost[a >> 20] > cost[b >> 20]; });
    len = std::max(len, v.size());
  }
  items.assign(len * NX, -1);
  for (int x = 0; x < NX; ++x)
    for (size_t j = 0; j < q[x].size(); ++j) items[j * NX + x] = q[x][j];
  return items;
}

extern "C" int encdiff_wgrad_group_plan(const EncdiffGemmArgs* probs, int n, float* workspace, long ws_floats,
                                        int* counters, int n_counters, void* blob, long capacity, long* blob_bytes) {
  if (!probs || n <= 0 || n > 2047 || !blob_bytes || ws_floats < 0 || n_counters < 0) return ENCDIFF_ERR_ARG;
  if ((uintptr_t)workspace & 127) return ENCDIFF_ERR_ARG;
  std::vector<WgProb> w((size_t)n);
  std::vector<double> cost((size_t)n);
  WgScratch sc{workspace, workspace ? ws_floats : 0, 0, counters, counters ? n_counters : 0, 0};
  for (int i = 0; i < n; ++i) {
    std::memset(&w[i], 0, sizeof(WgProb));
    const int rc = wg_prepare(probs[i], w[i], cost[i], sc);
    if (rc != ENCDIFF_OK) return rc;
    if (w[i].nblk <= 0 || w[i].nblk >= (1 << 20)) return ENCDIFF_ERR_SHAPE;
  }
  const std::vector<int> items = wg_items(w, cost);
  if (items.size() >= (size_t)1 << 30) return ENCDIFF_ERR_SHAPE;
  const long probs_off = (long)((sizeof(WgBlobHead) + 63) & ~(size_t)63);
  const long items_off = probs_off + (long)(sizeof(WgProb) * (size_t)n);
  const long bytes = items_off + (long)items.size() * 4;
  *blob_bytes = bytes;
  if (!blob) return ENCDIFF_OK;
  if (capacity < bytes || ((uintptr_t)blob & 7)) return ENCDIFF_ERR_ARG;
  char* out = (char*)blob;
  WgBlobHead h{};
  h.magic = WGG_MAGIC;
  h.n_probs = n;
  h.n_items = (int)items.size();
  h.lds = (int)WGG_LDS;
  h.probs_off = probs_off;
  h.items_off = items_off;
  h.bytes = bytes;
  std::memset(out, 0, (size_t)probs_off);
  std::memcpy(out, &h, sizeof(h));
  std::memcpy(out + probs_off, w.data(), sizeof(WgProb) * (size_t)n);
  std::memcpy(out + items_off, items.data(), items.size() * 4);
  return ENCDIFF_OK;
}

extern "C" int encdiff_wgrad_group_launch(const void* host_blob, const void* dev_blob, void* stream) {
  if (!host_blob || !dev_blob) return ENCDIFF_ERR_ARG;
  WgBlobHead h;
  std::memcpy(&h, host_blob, sizeof(h));
  if (h.magic != WGG_MAGIC || h.n_items <= 0 || h.lds > HALO_LDS_MAX) return ENCDIFF_ERR_ARG;
  static const hipError_t attr_ok = hipFuncSetAttribute((const void*)wgrad_group_kernel,
                                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)WGG_LDS);
  if (attr_ok != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)attr_ok;
  const char* d = (const char*)dev_blob;
  hipLaunchKernelGGL(wgrad_group_kernel, dim3((unsigned)h.n_items), dim3(256), (size_t)h.lds, (hipStream_t)stream,
                     (const WgProb*)(d + h.probs_off), (const int*)(d + h.items_off));
  const hipError_t e = hipGetLastError();
  return e != hipSuccess ? ENCDIFF_ERR_LAUNCH - (int)e : ENCDIFF_OK;
}

extern "C" int encdiff_gemm(const EncdiffGemmArgs* pa, void* stream) {
  if (pa && pa->dtype == ENCDIFF_DT_F32) return ed_gemm_f32(pa, (hipStream_t)stream);
  if (pa && pa->dtype != ENCDIFF_DT_BF16) return ENCDIFF_ERR_ARG;
  GemmPlan g;
  const int rc = prepare(pa, g);
  if (rc != ENCDIFF_OK) return rc;
  return launch_one(g, (hipStream_t)stream);
}

extern "C" int encdiff_gemm_ex(const EncdiffGemmArgs* pa, int defer_finalize, int* planned, void* stream) {
  if (planned) *planned = 0;
  if (!defer_finalize || (pa && pa->dtype == ENCDIFF_DT_F32)) return encdiff_gemm(pa, stream);
  GemmPlan g;
  const int rc = prepare(pa, g);
  if (rc != ENCDIFF_OK) return rc;
  if (!g.ws_path || g.fold) return launch_one(g, (hipStream_t)stream);
  GemmPlan t = g;
  t.ws_path = false;  // tile kernel only: the slabs wait for the consumer
  const int r = launch_one(t, (hipStream_t)stream);
  if (r == ENCDIFF_OK && planned) *planned = 1;
  return r;
}

// encdiff_gemm_pair_ex / encdiff_gemm_pair_dx: defer_d skips the input gradient's finalize
// (*dd = 1 when it had one to skip)
static int gemm_pair_impl(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad,
                          const EncdiffGemmArgs* prev_wgrad, int defer, bool defer_d, int* dd, void* stream) {
  *dd = 0;
  GemmPlan g1, g2, gp;
  int rc = prepare(wgrad, g1);
  if (rc != ENCDIFF_OK) return rc;
  rc = prepare(dgrad, g2);
  if (rc != ENCDIFF_OK) return rc;
  bool have_prev = false;
  if (prev_wgrad) {
    rc = prepare(prev_wgrad, gp);
    if (rc != ENCDIFF_OK) return rc;
    have_prev = gp.ws_path;
  }
  hipStream_t s = (hipStream_t)stream;
  hipError_t e;
  const int a1 = g1.p.a_mode, b1 = g1.p.b_mode, a2 = g2.p.a_mode, b2 = g2.p.b_mode;
  const bool lin = a1 == ENCDIFF_OPA_ROWM && b1 == ENCDIFF_OPB_ROWN && a2 == ENCDIFF_OPA_ROWK && b2 == ENCDIFF_OPB_ROWN;
  const bool conv = a1 == ENCDIFF_OPA_ROWM && b1 == ENCDIFF_OPB_IM2COL && a2 == ENCDIFF_OPA_IM2COL &&
                    b2 == ENCDIFF_OPB_CONV_DGRAD;
  // both split-K problems need disjoint slabs
  if (g1.ws_path && g2.ws_path && g1.p.workspace == g2.p.workspace) return ENCDIFF_ERR_ARG;
  const bool defer1 = defer && g1.ws_path;
  const bool dslabs = g2.ws_path && !g2.fold;  // the input gradient has a finalize pass
  auto run_g2 = [&]() -> int {  // input gradient alone, its finalize unless deferred
    if (defer_d && dslabs) {
      GemmPlan t = g2;
      t.ws_path = false;
      const int r = launch_one(t, s);
      if (r == ENCDIFF_OK) *dd = 1;
      return r;
    }
    return launch_one(g2, s);
  };
  if (g1.tile == 36) {  // WGL weight gradient (+ input gradient, + previous finalize)
    const EncdiffGemmArgs& pf = have_prev ? gp.user : g1.user;
    const int nf = have_prev ? fin_blocks(gp.user) : 0;
    const bool paired = wglpair_ok(g1, g2);
    e = paired ? wglpair_launch(g1, g2, pf, nf, s) : wgl_launch(g1.p, pf, nf, s);
    if (e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
    if (g1.ws_path && !defer1 && (e = launch_finalize(g1.user, s)) != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
    if (!paired) return run_g2();
    if (defer_d && dslabs) {
      *dd = 1;
      return ENCDIFF_OK;
    }
    if (g2.ws_path && (e = launch_finalize(g2.user, s)) != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
    return ENCDIFF_OK;
  }
  if (g1.tile >= 32 && g1.tile <= 34) {
    const EncdiffGemmArgs& pf = have_prev ? gp.user : g1.user;
    const int nf = have_prev ? fin_blocks(gp.user) : 0;
    if (wg3pair_ok(g1, g2)) {  // WG3 + input gradient + previous finalize in one grid
      e = wg3pair_launch(g1, g2, pf, nf, s);
      if (e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
      const bool f1 = g1.ws_path && !defer1, f2 = dslabs && !defer_d;
      if (f1 && (e = launch_finalize(g1.user, s)) != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
      if (f2 && (e = launch_finalize(g2.user, s)) != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
      if (dslabs && defer_d) *dd = 1;
      return ENCDIFF_OK;
    }
    // WG3 weight gradient (+ the previous finalize riding along), then the input gradient
    e = wg3_launch(g1.p, g1.tile, pf, nf, s);
    if (e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
    if (g1.ws_path && !defer1 && (e = launch_finalize(g1.user, s)) != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
    return run_g2();
  }
  if ((!lin && !conv) || (g1.tile != 4 && g1.tile != 5 && g1.tile != 7 && g1.tile != 9 && g1.tile != 10)) {
    // pairs the fused kernel does not cover
    if (have_prev && (e = launch_finalize(gp.user, s)) != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
    GemmPlan w = g1;
    w.ws_path = g1.ws_path && !defer1;
    rc = launch_one(w, s);
    return rc != ENCDIFF_OK ? rc : run_g2();
  }
  const EncdiffGemmArgs pf = have_prev ? gp.user : g1.user;
  const int nf = have_prev ? fin_blocks(gp.user) : 0;
  e = lin ? launch_pair_tiles<A_ROWM, B_ROWN, A_ROWK, B_ROWN>(g1, g2, pf, nf, s)
          : launch_pair_tiles<A_ROWM, B_IM2COL, A_IM2COL, B_CONVD>(g1, g2, pf, nf, s);
  if (e != hipSuccess) return ENCDIFF_ERR_LAUNCH - (int)e;
  const bool f1 = g1.ws_path && !defer1;
  const bool f2 = dslabs && !defer_d;
  if (dslabs && defer_d) *dd = 1;
  if (f1 && f2) {
    const int n1 = fin_blocks(g1.user), n2 = fin_blocks(g2.user);
    hipLaunchKernelGGL(gemm_finalize2_kernel, dim3((unsigned)(n1 + n2)), dim3(256), 0, s, g1.user, g2.user, n1);
    e = hipGetLastError();
  } else if (f1) {
    e = launch_finalize(g1.user, s);
  } else if (f2) {
    e = launch_finalize(g2.user, s);
  } else {
    e = hipGetLastError();
  }
  return e != hipSuccess ? ENCDIFF_ERR_LAUNCH - (int)e : ENCDIFF_OK;
}

extern "C" int encdiff_gemm_pair_ex(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad,
                                    const EncdiffGemmArgs* prev_wgrad, int defer, void* stream) {
  int dd;
  return gemm_pair_impl(wgrad, dgrad, prev_wgrad, defer, false, &dd, stream);
}

extern "C" int encdiff_gemm_pair_dx(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad,
                                    const EncdiffGemmArgs* prev_wgrad, int defer, int defer_dgrad, int* dgrad_deferred,
                                    void* stream) {
  int dd = 0;
  const int rc = gemm_pair_impl(wgrad, dgrad, prev_wgrad, defer, defer_dgrad != 0, &dd, stream);
  if (dgrad_deferred) *dgrad_deferred = rc == ENCDIFF_OK ? dd : 0;
  return rc;
}

extern "C" int encdiff_gemm_pair(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad, void* stream) {
  return encdiff_gemm_pair_ex(wgrad, dgrad, nullptr, 0, stream);
}

extern "C" int encdiff_gemm_finalize(const EncdiffGemmArgs* args, void* stream) {
  GemmPlan g;
  const int rc = prepare(args, g);
  if (rc != ENCDIFF_OK) return rc;
  if (!g.ws_path || g.fold) return ENCDIFF_OK;  // folded GEMMs combined their slabs in the kernel
  const hipError_t e = launch_finalize(g.user, (hipStream_t)stream);
  return e != hipSuccess ? ENCDIFF_ERR_LAUNCH - (int)e : ENCDIFF_OK;
}

extern "C" int encdiff_version(void) { return 1; }
