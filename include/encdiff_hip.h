/*
 * encdiff_hip.h -- C-ABI of libencdiff_hip.so, the MI355X (gfx950) kernels of the
 * EncDiff denoising path.
 *
 * The reference (SelenaGeRuiqi/EncDiff) has no FFI: its hot path is PyTorch eager
 * ops inside ldm/modules/diffusionmodules/openaimodel_enc.py, ldm/modules/attention.py,
 * ldm/models/diffusion/ddpm_enc.py and ldm/models/diffusion/ddim.py.  Each entry point
 * below names the reference computation it replaces (file:line).  The Python
 * module-level mirror of the reference API (encdiff_amd/ldm/...) calls these
 * through ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Caller owns all memory: device pointers + leading dimensions (in elements).
 *    The library never allocates.
 *  - Stream ordered: every launch goes on the `stream` argument (a hipStream_t,
 *    e.g. torch.cuda.current_stream().cuda_stream); no implicit synchronisation,
 *    so every call is hipGraph-capturable.
 *  - Errors: 0 on success, a negative ENCDIFF_ERR_* on bad arguments, and
 *    ENCDIFF_ERR_LAUNCH - hipError_t on a launch failure.
 *  - Threading: reentrant, no global mutable state.
 *  - Layout: activations are [rows][channels] bf16 (NHWC for images, token-major
 *    for transformer tokens) with a row stride `ld`; statistics / master weights /
 *    gradients are fp32.
 *  - dtype: the GEMM, GroupNorm, LayerNorm, attention and elementwise args carry a `dtype`
 *    field.  ENCDIFF_DT_BF16 (0, the default) is the product path above.  ENCDIFF_DT_F32
 *    runs the same entry point on fp32 activations (every bf16 operand / output named in
 *    the struct becomes fp32), forward AND backward: the reference's precision
 *    (main_val.py:525), so the denoiser's output and gradients can be held to the fp32
 *    tolerance.  Supported there: GEMM OPA_ROWK x OPB_ROWK / OPB_ROWN, OPA_IM2COL (resample
 *    NONE / UP2) x OPB_ROWK / OPB_CONV_DGRAD, OPA_ROWM x OPB_ROWN / OPB_IM2COL (+ bias_grad)
 *    into OUT_F32 / OUT_F32_ACCUM (alpha, bias, fp32 resid; no split-K / epilogue
 *    statistics); GroupNorm fwd / bwd (FiLM, SiLU, resid, accumulate) without in_stats /
 *    x_from; LayerNorm fwd / bwd (c <= 512, no dy_from); attention fwd / bwd dh in
 *    {8, 16, 32, 64} (no fp8); elementwise COPY, SILU, SILU_BWD, GEGLU, GEGLU_BWD, ADD,
 *    RESAMPLE, RESAMPLE_BWD.  Other combinations return ENCDIFF_ERR_UNSUPPORTED.
 */
#ifndef ENCDIFF_HIP_H
#define ENCDIFF_HIP_H

#ifdef __cplusplus
extern "C" {
#endif

#define ENCDIFF_OK 0
#define ENCDIFF_ERR_ARG (-1)
#define ENCDIFF_ERR_SHAPE (-2)
#define ENCDIFF_ERR_UNSUPPORTED (-3)
#define ENCDIFF_ERR_LAUNCH (-1000)

enum { ENCDIFF_DT_BF16 = 0, ENCDIFF_DT_F32 = 1 };

/* ---------------------------------------------------------------- GEMM / conv
 * C[M][N] = alpha * sum_k A[m][k] * B[k][n]  (+ bias[n]) (+ resid[m][n])
 * Replaces every nn.Linear / 1x1 Conv2d / 3x3 Conv2d forward and backward on the
 * path: openaimodel_enc.py:204,230,237-241,508-512,521,687 (conv/linear),
 * attention.py:159-167,43,58 (q/k/v/out, GEGLU, FF), attention.py:233-259 (proj_in/out).
 */
enum {
  ENCDIFF_OPA_ROWK = 0,   /* A[m][k] at a + m*lda + k                                  */
  ENCDIFF_OPA_IM2COL = 1, /* A[m][k] = im2col3x3(src)[pixel m][tap*cin + c] (conv fwd / dgrad) */
  ENCDIFF_OPA_ROWM = 2    /* A stored transposed: A[m][k] at a + k*lda + m (wgrad of dY)   */
};
enum {
  ENCDIFF_OPB_ROWK = 0,       /* B[k][n] at b + n*ldb + k (weights [out][in])               */
  ENCDIFF_OPB_ROWN = 1,       /* B[k][n] at b + k*ldb + n                                    */
  ENCDIFF_OPB_CONV_DGRAD = 2, /* B[(tap,co)][ci] = Wf[co][T-1-tap][ci], Wf packed [co][T][cin], T = 9
                                 (16 with resample K4S2_T)                                     */
  ENCDIFF_OPB_IM2COL = 3      /* B[pixel][tap*cin + c] = im2col3x3(src) (conv wgrad)          */
};
enum {
  ENCDIFF_OUT_BF16 = 0,
  ENCDIFF_OUT_F32 = 1,
  ENCDIFF_OUT_F32_ATOMIC = 2,       /* atomicAdd into fp32 C (split-K / grad accumulate)   */
  ENCDIFF_OUT_F32_ATOMIC_CONVW = 3, /* atomicAdd, column n=(tap,ci) scattered to the reference
                                       Conv2d weight layout [co][ci][3][3]                   */
  ENCDIFF_OUT_F32_ACCUM = 4,        /* fp32 C += result, single writer per element (weight
                                       gradients): with split_k > 1 the slabs are summed in a
                                       fixed order -> bitwise reproducible                   */
  ENCDIFF_OUT_BF16_GEGLU = 5,       /* GEGLU proj (attention.py GEGLU): C = f [M][N] bf16 (N = 2*inner,
                                       +bias) and aux = y [M][N/2] = f[:, :N/2] * gelu(f[:, N/2:])
                                       from the bf16-rounded f; OPA_ROWK x OPB_ROWK, split_k 1   */
  ENCDIFF_OUT_BF16_GEGLU_BWD = 6    /* GEGLU backward fused into the dgrad producing dy [M][N]
                                       (N = inner): aux = f [M][2N] input, C = df [M][2N] bf16
                                       (d of the value half, d of the gate half); split_k 1   */
};
enum {
  ENCDIFF_RESAMPLE_NONE = 0,
  ENCDIFF_RESAMPLE_DOWN2 = 1, /* source is (2h,2w); AvgPool2d(2) on the fly  (openaimodel_enc.py:156) */
  ENCDIFF_RESAMPLE_UP2 = 2,   /* source is (h/2,w/2); nearest x2 on the fly (openaimodel_enc.py:116) */
  ENCDIFF_RESAMPLE_STRIDE2 = 3, /* source is (2h,2w); 3x3 taps at (2y+ky, 2x+kx), zero pad right/bottom
                                  only: F.pad(x,(0,1,0,1)) + Conv2d(k3, s2, p0) (model.py Downsample) */
  ENCDIFF_RESAMPLE_K4S2 = 4,   /* source is (2h,2w); 4x4 taps (K = 16*cin) at (2y+ky-1, 2x+kx-1):
                                  Conv2d(k4, s2, p1) of Encoder4 (openaimodel_enc.py:1002-1009)   */
  ENCDIFF_RESAMPLE_K4S2_T = 5, /* input gradient of K4S2: source dY is (h/2,w/2); with
                                  OPB_CONV_DGRAD (16 taps, flipped) computes dX at (h,w)          */
  ENCDIFF_RESAMPLE_K4S2_TP = 6 /* the same input gradient by output parity: K = 4*cin (the 2x2 taps
                                  that reach each parity class of (y, x)), M = batch*h*w with
                                  batch*h*w/4 % 128 == 0; rows are computed parity-major and
                                  written to their pixel.  OPB_CONV_DGRAD only, no atomic c_mode  */
};

typedef struct EncdiffConvGeom {
  int batch;     /* images                                                       */
  int h, w;      /* spatial size of the conv input after resampling (== output)  */
  int cin;       /* channels of the im2col source                                */
  int resample;  /* ENCDIFF_RESAMPLE_*                                           */
  int pad_;
  long ld_src;   /* pixel stride of the source tensor, elements                  */
} EncdiffConvGeom;

typedef struct EncdiffGemmArgs {
  int M, N, K;
  int a_mode, b_mode, c_mode;
  const void* a; long lda;   /* bf16 */
  const void* b; long ldb;   /* bf16 */
  void* c; long ldc;         /* bf16 or fp32 per c_mode */
  EncdiffConvGeom conv;      /* for IM2COL operands                                */
  int conv_cout;             /* OPB_CONV_DGRAD: forward conv's output channels     */
  int convw_cin;             /* OUT_F32_ATOMIC_CONVW: forward conv's input channels */
  float alpha;
  int split_k;               /* >= 1; > 1 needs an atomic c_mode or a workspace     */
  const float* bias;         /* [N] fp32 or NULL                                   */
  const void* resid; long ld_resid;  /* bf16 [M][N] or NULL                        */
  float* bias_grad;          /* OPA_ROWM only: += sum_k A[m][k] into bias_grad[m]  */
  int tile;                  /* 0 = auto, else 1:128x128 2:128x64 3:64x128 4:64x64, 5:64x64 with a
                                4-deep LDS ring, 6:64x128 with a 3-deep ring, 7:64x64 and
                                8:64x128 with 128-deep k stages (others: 64), 9 / 10: 64x64 with a
                                6- / 8-deep ring (96 / 128 KB of LDS: a short split's k-tiles all
                                in flight at once), 16-23: halo tiles (implicit im2col only), 32-34:
                                3x3 conv weight gradient kernel WG3 (OPA_ROWM x OPB_IM2COL, resample
                                NONE / UP2, h == w in {4, 8, 16}, M % 32 == 0, cin % 16 == 0; split_k =
                                chunks of whole images, each chunk one fp32 slab): workgroups of 32 couts
                                x 16 cins x 9 taps whose waves split the chunk's pixels; 32 shares one
                                grid with the layer's input gradient in encdiff_gemm_pair_ex, 34 never
                                pairs, 33 uses 8-wave workgroups; 36: linear weight gradient kernel WGL
                                (OPA_ROWM x OPB_ROWN, M % 64 == 0, N % 64 == 0, K % (split_k*128) == 0;
                                64 x 64 output parts, waves split each chunk's tokens), paired with the
                                input gradient in encdiff_gemm_pair_ex */
  int dtype;                 /* ENCDIFF_DT_BF16 (a, b, resid and BF16 outputs bf16) or ENCDIFF_DT_F32 */
  float* workspace;          /* split_k > 1 with a BF16/F32/F32_ACCUM c_mode: fp32 scratch of split_k*M*N
                                (+ split_k*M when bias_grad is set: per-split bias-gradient slabs);
                                each split writes its own [M][N] slab, a finalize pass sums the
                                slabs in order (reproducible) and applies alpha/bias/resid    */
  void* aux; long ld_aux;    /* GEGLU c_modes: y output (BF16_GEGLU) / f input (BF16_GEGLU_BWD)  */
  float* gn_stats; long ld_gn_stats;  /* optional, OUT_BF16 with split_k 1 and M % 64 == 0: per
                                64-row segment s and column n, the sum and sum of squares of the
                                bf16 outputs at gn_stats[(2s)*ld + n] and [(2s+1)*ld + n] -- the
                                GroupNorm statistics of the tensor this GEMM produces, so that
                                encdiff_groupnorm_fwd needs no reduction pass (in_stats)       */
  const float* ln_gamma;     /* optional LayerNorm of the produced rows (attention.py norm1/2/3): */
  const float* ln_beta;      /*   OUT_BF16, split_k 1, the tile spans all N columns (N <= 128);   */
  void* ln_y; long ld_ln_y;  /*   ln_y = LN(C) bf16 from the stored bf16 C, two-pass fp32 stats,   */
  float* ln_stats;           /*   ln_stats [M][2] (mean, rstd) for the backward                  */
  float ln_eps;
  int pad3_;
  int* split_counters;       /* optional, split_k > 1 with a workspace (not OPA_ROWM, not K4S2_TP,
                                N % 8 == 0): the splits combine IN the kernel -- the last split
                                to finish a tile (one int ticket per output tile, zero on entry,
                                left zero) sums the tile's slabs in split order (reproducible)
                                and applies alpha/bias/resid; no finalize pass.  NULL: finalize */
  /* optional (agn_gamma != NULL), forward 3x3 convolutions OPA_IM2COL x OPB_ROWK (resample NONE /
     UP2, OUT_BF16, tile 0 or 4): the A operand is GroupNorm32(+FiLM)(+SiLU) of the im2col source x
     -- ResBlock in_layers / out_layers (openaimodel_enc.py:201-205, 225-232, 267-271; util.py:242-244)
     -- applied to each staged tile in LDS, so the normalised activation never goes to memory.  Every
     workgroup computes the statistics (fp32 sum / sum of squares per (image, group), 32 groups) of
     the images its output rows read, from x itself: x must be complete (no deferred slabs).
     Replaces the encdiff_groupnorm_fwd launch in front of the conv where nothing saves its output
     (sampling / inference). */
  const float* agn_gamma;
  const float* agn_beta;     /* [cin] */
  const float* agn_film;     /* optional fp32 [batch][ld_agn_film]: scale at [c], shift at [cin + c] */
  long ld_agn_film;
  float agn_eps;
  int agn_silu;
  /* optional (lna_gamma != NULL), linear forwards OPA_ROWK x OPB_ROWK (bf16 / GEGLU output, tile 0
     or 4, split 1, K <= 1024, K % 8 == 0): the A operand is LayerNorm(A) over its K channels --
     BasicTransformerBlock norm1 / norm2 / norm3 (attention.py:210-230) -- applied to each staged
     tile in LDS.  Every workgroup reduces the mean / rstd (fp32, one pass) of its rows from A in a
     prologue.  Replaces the encdiff_layernorm_fwd launch in front of the linear where nothing
     saves the normalised rows (sampling / inference). */
  const float* lna_gamma;
  const float* lna_beta;     /* [K] */
  float lna_eps;
} EncdiffGemmArgs;

int encdiff_gemm(const EncdiffGemmArgs* args, void* stream);

/* Two independent GEMMs of one layer's backward in ONE launch: the weight gradient
 * (a_mode OPA_ROWM) and the input gradient (linear: OPA_ROWK x OPB_ROWN; 3x3 conv:
 * OPA_IM2COL x OPB_CONV_DGRAD), their split-K finalizes in one more.  Results are
 * identical to two encdiff_gemm calls; pairs outside these forms run as two calls.  When
 * both use split-K their workspaces must be distinct.  Replaces the autograd backward of
 * one nn.Linear / nn.Conv2d (openaimodel_enc.py:230,237-241; attention.py:159-167,43,58). */
int encdiff_gemm_pair(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad, void* stream);

/* encdiff_gemm_pair with deferred weight-gradient finalizes.  defer != 0: when `wgrad` uses
 * split-K slabs its finalize (C += ordered slab sum, + bias gradient) is NOT launched; the
 * caller hands `wgrad` to a later call as `prev_wgrad`, whose launch then runs that finalize
 * in extra workgroups (or to encdiff_gemm_finalize).  Its slabs must stay untouched until
 * then (the next pair uses a different workspace region).  Results are identical. */
int encdiff_gemm_pair_ex(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad,
                         const EncdiffGemmArgs* prev_wgrad, int defer, void* stream);

/* encdiff_gemm_pair_ex that may also defer the INPUT gradient's finalize: defer_dgrad != 0 and
 * `dgrad` leaves split-K slabs for a finalize pass -> that pass is not launched and
 * *dgrad_deferred = 1; the caller hands `dgrad` to its consumer (EncdiffGroupNormArgs.x_from of
 * a GroupNorm backward) or to encdiff_gemm_finalize before the workspace half is reused.
 * Otherwise *dgrad_deferred = 0 and the result is encdiff_gemm_pair_ex's. */
int encdiff_gemm_pair_dx(const EncdiffGemmArgs* wgrad, const EncdiffGemmArgs* dgrad,
                         const EncdiffGemmArgs* prev_wgrad, int defer, int defer_dgrad, int* dgrad_deferred,
                         void* stream);

/* Grouped weight gradients: n weight-gradient GEMMs (a_mode OPA_ROWM, b_mode OPB_ROWN or
 * OPB_IM2COL, c_mode OUT_F32 / OUT_F32_ACCUM, optional bias_grad) in ONE launch (split_k /
 * workspace / tile of the problems are ignored).  Replaces the autograd weight gradients of every
 * nn.Linear / nn.Conv2d of a backward region (openaimodel_enc.py:230, 237-241, 255-275;
 * attention.py:159-167, 211-261) once their dY tensors exist.  Deep problems are cut into chunks
 * whose fp32 partials go to `workspace` (ws_floats floats, 16-byte aligned, this group's alone
 * while it runs) and are combined in the kernel by the chunk that finishes last (one ticket per
 * output part in `counters`, n_counters zeroed ints, left zero); every output element is one sum
 * in a fixed order, so results are reproducible run to run.  workspace / counters NULL: every
 * problem runs whole.
 * encdiff_wgrad_group_plan validates the problems and writes the launch description into `blob`
 * (8-byte aligned host memory of `capacity` bytes; blob == NULL: only *blob_bytes is set).  The
 * caller copies the blob byte for byte into device memory it owns and keeps (a captured graph
 * reads it at every replay), then encdiff_wgrad_group_launch(host copy, device copy, stream)
 * enqueues the grid.  Every pointer inside the problems, the workspace and the counters must
 * stay valid for as long as the blob is launched. */
int encdiff_wgrad_group_plan(const EncdiffGemmArgs* probs, int n, float* workspace, long ws_floats, int* counters,
                             int n_counters, void* blob, long capacity, long* blob_bytes);
int encdiff_wgrad_group_launch(const void* host_blob, const void* dev_blob, void* stream);

/* The split-K finalize of a GEMM launched with a deferred finalize (no-op without slabs). */
int encdiff_gemm_finalize(const EncdiffGemmArgs* args, void* stream);

/* encdiff_gemm with an optional deferred finalize.  defer_finalize != 0 and the plan keeps
 * split-K slabs without combining them in the kernel: only the tile kernel is launched and
 * *planned (if non-NULL) is set to 1; the caller then hands `args` to the consumer that
 * combines the slabs (EncdiffGroupNormArgs.x_from) or to encdiff_gemm_finalize before anything
 * else touches the workspace or C.  Otherwise identical to encdiff_gemm (*planned = 0).
 * Replaces the same nn.Conv2d / nn.Linear forward as encdiff_gemm. */
int encdiff_gemm_ex(const EncdiffGemmArgs* args, int defer_finalize, int* planned, void* stream);

/* ---------------------------------------------------------------- GroupNorm
 * y = act( GN(x) * (1 + scale[b,c]) + shift[b,c] )
 * Replaces GroupNorm32 + SiLU (+ FiLM) of ResBlock in/out_layers and UNet.out
 * (openaimodel_enc.py:201-205,225-232,267-271,684-686; util.py:242-244) and the
 * SpatialTransformer Normalize (attention.py:76-77, eps 1e-6, no act).
 */
typedef struct EncdiffGroupNormArgs {
  int batch, hw, c, groups;
  float eps;
  int silu;                  /* apply SiLU after the affine/FiLM                   */
  const void* x; long ldx;   /* bf16 [batch*hw][c]                                 */
  const float* gamma;
  const float* beta;
  const float* film; long ld_film;   /* optional fp32 [batch][ld_film]: scale at [c], shift at [C + c] */
  void* y; long ldy;         /* bf16 out                                           */
  float* stats;              /* fp32 [batch][groups][2] (mean, rstd)               */
  /* backward only */
  const void* dy; long lddy;
  void* dx; long lddx;       /* bf16                                                */
  int accumulate_dx;         /* dx += result                                        */
  int dtype;                 /* ENCDIFF_DT_F32: every activation / gradient fp32    */
  float* dgamma_part;        /* fp32 [batch][ld_part] per-image partial sums (reduced later) */
  float* dbeta_part;
  long ld_part;
  float* dfilm; long ld_dfilm;       /* fp32 [batch][ld_dfilm]: dscale at [c], dshift at [C + c] */
  const void* resid; long ld_resid;  /* backward: optional bf16 residual-branch gradient added to dx */
  const float* in_stats; long ld_in_stats;  /* forward, optional: per-64-row-segment channel sums
                                of x written by its producer GEMM (EncdiffGemmArgs.gn_stats; hw
                                a multiple of 64): the statistics come from them, x is read once */
  const EncdiffGemmArgs* x_from;  /* forward, optional (bf16, no in_stats): x is the output of this
                                GEMM, launched by encdiff_gemm_ex with its split-K finalize deferred
                                (bf16 C == x, ldc == ldx, N == c, M == batch*hw): the kernel sums
                                the slabs in the finalize's order, applies alpha / bias / resid,
                                WRITES x (bitwise the finalize's result) and normalises it -- one
                                launch instead of finalize + GroupNorm.  Backward: the same for dy
                                (C == dy, ldc == lddy; e.g. the input gradient of the conv that read
                                this GroupNorm's output, its finalize deferred by
                                encdiff_gemm_pair_dx) */
  /* backward, optional (bf16, no x_from): dy / resid are given at the resolution of a 2x resample
     (ENCDIFF_RESAMPLE_DOWN2 avg-pool / UP2 nearest) that follows this GroupNorm -- its output feeds
     the downsampling / upsampling conv of a ResBlock, or the ResBlock's skip branch resamples x
     (openaimodel_enc.py:248-253, 264-265) -- and the kernel reads them through that resample's
     adjoint (dy: rounded to bf16 as the adjoint pass would store it; resid: added after dx's own
     rounding, as an accumulating adjoint pass would): two elementwise launches fewer per ResBlock.
     w: the image width at this GroupNorm's resolution (hw = h * w), needed with either mode. */
  int dy_resample, resid_resample;
  int w, pad_rs_;
  /* optional (bf16, silu): the SiLU gradient at z, silu'(z) = s (1 + z (1 - s)), s = sigmoid(z), one
     bf16 [batch*hw][c] row per pixel (ld_dsilu): the training forward writes it beside y, the backward
     reads it instead of recomputing z's two transcendentals per element (its VALU-bound pass 1) */
  void* dsilu; long ld_dsilu;
  /* backward, optional: a device weight-gradient plan of encdiff_st_wgrad_plan whose chunk fold rides
     in this launch as fold_blocks extra workgroups after the GroupNorm's (encdiff_st_wgrad_launch_nofold
     launched its grid before; the fold is off the GroupNorm's critical path) -- one launch fewer per
     fused transformer block */
  const void* fold_plan; int fold_blocks, pad_fold_;
} EncdiffGroupNormArgs;

int encdiff_groupnorm_fwd(const EncdiffGroupNormArgs* args, void* stream);
int encdiff_groupnorm_bwd(const EncdiffGroupNormArgs* args, void* stream);

/* ---------------------------------------------------------------- LayerNorm
 * BasicTransformerBlock norm1/2/3 (attention.py:206-208, 211-215), eps 1e-5.
 */
typedef struct EncdiffLayerNormArgs {
  int rows, c;
  float eps;
  const void* x; long ldx;
  const float* gamma; const float* beta;
  void* y; long ldy;
  float* stats;              /* fp32 [rows][2] (mean, rstd) */
  const void* dy; long lddy; /* backward */
  void* dx; long lddx;
  int accumulate_dx;         /* dx += (residual branch)                            */
  float* dgamma_part;        /* fp32 [parts][ld_part]                              */
  float* dbeta_part;
  long ld_part;
  int parts;                 /* number of partial rows (grid size of the backward) */
  int dtype;                 /* ENCDIFF_DT_F32: every activation / gradient fp32    */
  const void* resid; long ld_resid; /* backward: optional bf16 residual-branch gradient:
                                        dx = resid + LN_bwd (out of place; may alias dx) */
  const EncdiffGemmArgs* dy_from;   /* backward, optional: dy is the output of this GEMM whose
                                        split-K finalize was deferred (encdiff_gemm_pair_dx; bf16
                                        C == dy, ldc == lddy, N == c, M == rows): its slabs are
                                        combined here as the finalize would, dy written, as
                                        EncdiffGroupNormArgs.x_from */
} EncdiffLayerNormArgs;

int encdiff_layernorm_fwd(const EncdiffLayerNormArgs* args, void* stream);
int encdiff_layernorm_bwd(const EncdiffLayerNormArgs* args, void* stream);

/* ---------------------------------------------------------------- Attention
 * softmax(q k^T * dh^-0.5) v per head, q/k/v/o as [rows][ld] with head h at
 * columns [h*dh, (h+1)*dh) ('b n (h d)', attention.py:170-193).  Self-attention
 * (keys = the same tokens) and cross-attention to the concept tokens (keys = 20).
 * dh in {8, 16, 32, 64} (fwd + bwd), 128 (fwd only: the VQ encoder's AttnBlock);
 * ENCDIFF_ERR_SHAPE when a head group's K/V tiles exceed one workgroup's LDS.
 */
typedef struct EncdiffAttnArgs {
  int batch, heads, sq, sk, dh;
  float scale;
  const void* q; long ldq;
  const void* k; long ldk;
  const void* v; long ldv;
  void* o; long ldo;
  float* lse;                /* fp32 [batch*heads][sq] log-sum-exp (for backward)  */
  const void* d_o; long lddo;  /* backward */
  void* dq; long lddq;
  void* dk; long lddk;
  void* dv; long lddv;
  int fp8_qk;                /* 1: scores Q K^T on fp8 (OCP e4m3) MFMA, fwd and bwd recompute;
                                softmax, P V and the gradient products stay bf16 / fp32 */
  int dtype;                 /* ENCDIFF_DT_F32: q, k, v, o, d_o, dq, dk, dv fp32      */
} EncdiffAttnArgs;

int encdiff_attention_fwd(const EncdiffAttnArgs* args, void* stream);
int encdiff_attention_bwd(const EncdiffAttnArgs* args, void* stream);

/* ---------------------------------------------------------------- elementwise */
enum {
  ENCDIFF_EW_COPY = 0,        /* y = x                                               */
  ENCDIFF_EW_SILU = 1,        /* y = silu(x)                        (emb_layers[0]) */
  ENCDIFF_EW_SILU_BWD = 2,    /* y = dy * silu'(x)                                   */
  ENCDIFF_EW_GEGLU = 3,       /* y[:, j] = x[:, j] * gelu(x[:, n + j])  (attention.py:42-44) */
  ENCDIFF_EW_GEGLU_BWD = 4,   /* dx[:, j], dx[:, n+j] from dy and x                  */
  ENCDIFF_EW_ADD = 5,         /* y = x + x2                                          */
  ENCDIFF_EW_RESAMPLE = 6,    /* y = resample(x) (down: avgpool2, up: nearest2)      */
  ENCDIFF_EW_RESAMPLE_BWD = 7,/* y (+)= adjoint of resample applied to x             */
  ENCDIFF_EW_F32_TO_BF16 = 8,
  ENCDIFF_EW_BF16_TO_F32 = 9
};
typedef struct EncdiffEwArgs {
  int op;
  int rows, cols;            /* output logical shape [rows][cols]                  */
  const void* x; long ldx;
  const void* x2; long ldx2;
  void* y; long ldy;
  int accumulate;            /* y += result                                        */
  int resample;              /* ENCDIFF_RESAMPLE_* for RESAMPLE ops                */
  int batch, h, w;           /* output spatial dims for RESAMPLE ops               */
  int dtype;                 /* ENCDIFF_DT_F32: x, x2, y fp32                       */
} EncdiffEwArgs;

int encdiff_elementwise(const EncdiffEwArgs* args, void* stream);

/* ---------------------------------------------------------------- small convs
 * UNet input conv 3->64 (openaimodel_enc.py:521) and output conv 64->3
 * (openaimodel_enc.py:687): channel counts not multiples of 8.  NHWC bf16
 * activations, fp32 weights in the reference layout [co][ci][3][3].
 */
typedef struct EncdiffSmallConvArgs {
  int batch, h, w, cin, cout;
  const void* x; long ldx;        /* bf16 (or fp32 when x_f32)                     */
  int x_f32;                      /* input x is fp32 NCHW (the UNet input tensor) */
  const float* weight;            /* [cout][cin][3][3] fp32                        */
  const float* bias;
  void* y; long ldy;              /* bf16 NHWC, or fp32 NCHW when y_f32            */
  int y_f32;
  int pad_;
  /* backward */
  const void* dy; long lddy;      /* bf16 NHWC or fp32 NCHW (dy_f32)               */
  int dy_f32;
  int pad2_;
  void* dx; long lddx;            /* bf16 NHWC (or NULL)                           */
  float* dweight;                 /* fp32 atomic accumulate, reference layout      */
  float* dbias;
} EncdiffSmallConvArgs;

int encdiff_small_conv_fwd(const EncdiffSmallConvArgs* args, void* stream);
int encdiff_small_conv_bwd(const EncdiffSmallConvArgs* args, void* stream);

/* ---------------------------------------------------------------- diffusion
 * timestep_embedding (util.py:179-199) -> bf16 [batch][dim]
 */
int encdiff_timestep_embedding(const long long* t, int batch, int dim, float max_period,
                               void* out_bf16, void* stream);

/* The same embedding in fp32 [batch][dim] (the ENCDIFF_DT_F32 forward). */
int encdiff_timestep_embedding_f32(const long long* t, int batch, int dim, float max_period, float* out,
                                   void* stream);

/* fp32 layout change of the denoiser's input / output (the ENCDIFF_DT_F32 forward):
 * dir 0: x NCHW [batch][c][hw] -> y rows [batch*hw][ld], channels c..cpad-1 zero;
 * dir 1: x rows [batch*hw][ld] -> y NCHW (first c channels). */
int encdiff_nchw_rows_f32(const float* x, int batch, int c, int hw, int cpad, float* y, long ld, int dir,
                          void* stream);

/* q_sample (ddpm_enc.py:292-295): x_t = sqrt_ac[t] x0 + sqrt_1mac[t] eps.
 * x0, eps, x_t fp32 NCHW [batch][3*hw]. */
int encdiff_q_sample(const float* x0, const float* eps, const long long* t, const float* sqrt_ac,
                     const float* sqrt_1mac, int batch, int per_sample, float* x_t, void* stream);

/* The same with x0 = scale[0] * z: get_first_stage_encoding's scale_factor (ddpm_enc.py:775-783,
 * a device scalar) applied on the fly, so the scaled latent is never materialised. */
int encdiff_q_sample_scaled(const float* z, const float* scale, const float* eps, const long long* t,
                            const float* sqrt_ac, const float* sqrt_1mac, int batch, int per_sample, float* x_t,
                            void* stream);

/* p_losses L1 (ddpm_enc.py:1194-1213): loss_simple[b] = mean|eps - pred|,
 * out[0] = mean_b loss_simple (= loss with logvar 0), out[1] = mean_b lvlb[t_b] loss_simple[b];
 * grad_pred = sign(pred - eps) / (batch * per_sample) * l_simple_weight.
 * partials: caller scratch of `batch` floats (receives loss_simple[b]); counter: a
 * zero-initialised device uint32 the kernel leaves at zero (the last block folds the batch in a
 * fixed order: one launch, no memset, bitwise reproducible). */
int encdiff_l1_loss(const float* pred, const float* eps, const long long* t, const float* lvlb,
                    int batch, int per_sample, float l_simple_weight, float* out2, float* grad_pred,
                    float* partials, unsigned int* counter, void* stream);

/* DDIM update (ddim.py:197-206) for one step with scalar coefficients:
 * pred_x0 = (x - s1 e) / sqrt(a_t); x' = sqrt(a_prev) pred_x0 + sqrt(1-a_prev-sigma^2) e + sigma z. */
int encdiff_ddim_step(const float* x, const float* e, const float* noise, int n, float a_t,
                      float a_prev, float sigma, float sqrt_one_minus_at, float* x_prev, float* pred_x0,
                      void* stream);

/* Same update, coefficients read at execution time from a device table
 * coef[index][4] = {a_t, a_prev, sigma, sqrt(1 - a_t)} with `index` a device int --
 * one captured step graph replays the whole DDIM loop (ddim.py:135-162). The kernel
 * also decrements *index after the update when `advance` != 0. */
int encdiff_ddim_step_indexed(const float* x, const float* e, const float* noise, int n, const float* coef,
                              int* index, int advance, float* x_prev, float* pred_x0, void* stream);

/* ---------------------------------------------------------------- optimizer / EMA
 * Fused AdamW (torch defaults; ddpm_enc.py:1615) + optional LitEma update
 * (ema.py:25-44) over one flat fp32 parameter arena, plus the bf16 packing of
 * the updated weights into the compute layouts (pack table).
 */
/* hyper (device fp32[8], read at execution time so a captured step graph can be
 * replayed with a new lr / step): [lr, beta1, beta2, eps, weight_decay,
 * lr / (1 - beta1^step), 1 / sqrt(1 - beta2^step), ema (1 - decay)].
 * The EMA covers the first ema_n elements of the arena (the UNet parameters). */
int encdiff_adamw_ema(float* p, const float* g, float* m, float* v, float* ema, long long n,
                      const float* hyper, long long ema_n, void* stream);
/* encdiff_adamw_ema that also writes the updated weights as bf16 into `mirror` (n elements,
 * 8-byte aligned, index for index with p; NULL: none): the GEMM operand copies of every weight
 * whose compute layout is its arena layout, so no separate repack pass reads the arena again. */
int encdiff_adamw_ema_mirror(float* p, const float* g, float* m, float* v, float* ema, long long n,
                             const float* hyper, long long ema_n, void* mirror, void* stream);

/* Pack fp32 master weights into bf16 compute layouts.  Each job copies `rows x cols`
 * elements: dst[r*dst_ld + c] = src[src_index(r, c)], kind 0: src[r*cols + c]
 * (identity), kind 1: conv [co][ci][3][3] -> [co][tap][ci] (r=co, c=tap*cin+ci), kind 2:
 * conv [co][cin][taps] -> [co][tap][8] with channels cin..7 zero (cols = 8*taps; the
 * first Encoder4 conv, image channels padded to 8).  Split-bf16 (bf16x3) forms, hi = bf16(w),
 * lo = bf16(w - hi): kind 3: [co][tap][cin] -> [co][tap][hi|hi|lo] (cols = 3*cin*taps); kind 4:
 * [co][cin][taps] (cin <= 8) -> [co][tap][hi8|hi8|lo8] (cols = 24*taps); kind 5: [co][cin] ->
 * [co][hi|hi|lo|I|I] (cols = 5*cin, co == cin: a 1x1 conv plus an identity residual).  With
 * activations stored [hi|lo|hi] (+ [hi|lo] for the residual) one GEMM forms a_hi w_hi + a_lo w_hi +
 * a_hi w_lo: fp32-class products for the Encoder4 forward (see cond.py).  kind 6: the transpose,
 * src [rows][cols] -> dst [cols][rows] (a Linear's [in][out] copy: the B operands of the
 * SpatialTransformer backward kernels, encdiff_st_tail_bwd / encdiff_st_head_bwd). */
typedef struct EncdiffPackJob {
  long long src_off, dst_off;
  int rows, cols, kind, cin;
} EncdiffPackJob;
int encdiff_pack_weights(const float* src, void* dst_bf16, const EncdiffPackJob* jobs, int njobs,
                         void* stream);

/* Reduce per-part partial sums into the fp32 gradient arena:
 * grad[col_index[j]] += sum_{r < rows} part[r * ld + j], j < cols. */
int encdiff_reduce_partials(const float* part, long ld, int rows, int cols, const int* col_index,
                            float* grad, void* stream);

/* Fold a channel-padded conv weight gradient into the arena (the GEMM-computed weight gradient of
 * a conv whose narrow side is padded to `cpad` channels, openaimodel_enc.py:687 out conv and :521
 * input conv, Encoder4's first Conv2d :1002):
 *   gw[o][c][t] += dw[o][t][c],  o < co, c < cin <= cpad, t < taps   (dw rows: [taps][cpad])
 *   gb[o] += db[o]; db[o] = 0   (when db != NULL: a GEMM bias-gradient accumulator, left zero
 *                                for the next step -- graph-replay safe, no memset)
 * One launch; replaces torch permute/add and reduction kernels in the captured step. */
int encdiff_grad_fold(const float* dw, int co, int cin, int cpad, int taps, float* db, float* gw, float* gb,
                      void* stream);

/* ---------------------------------------------------------------- input path
 * GPU-resident dataset: uint8 images [n_images][h][w][c] (Shapes3D layout, disdata.py:45-97)
 * stay in HBM; one launch gathers a batch and applies ToTensor + Normalize(0.5, 0.5)
 * (disdata.py:82-88) and get_input's 'b h w c -> b c h w' float (ddpm_enc.py:347-353):
 *   out[b][ch][y][x] = (pool[id][y][x][ch] / 255 - 0.5) / 0.5,
 *   id = perm[(*step mod steps_per_epoch) * batch + b]          (shuffled epoch order)
 * perm: device int64 [steps_per_epoch * batch]; step: device int64 counter (NULL = 0),
 * advanced by one after the gather when `advance` != 0, so a captured step graph walks
 * the epoch by itself. */
int encdiff_gather_images_u8(const void* pool, long long n_images, int h, int w, int c,
                             const long long* perm, long long* step, int steps_per_epoch, int batch,
                             int advance, float* out, void* stream);

/* ---------------------------------------------------------------- concept encoder (§8(f) row 2)
 * Encoder4.warp (openaimodel_enc.py:1015-1041): `units` independent MLPs
 * u[:, i] -> Linear(1,64) -> ELU -> Linear(64,128) -> ELU -> Linear(128,context_dim),
 * out[:, i*context_dim + m].  fp32 throughout (the reference's precision).
 * params: unit i's tensors contiguous at params + i*unit_stride in nn.Sequential order
 * [W1 64][b1 64][W2 128x64][b2 128][W3 context_dim x 128][b3 context_dim] (the layout
 * of the parameter arena).  The backward ADDS the weight gradients into `grads` (same
 * layout) and writes du: one workgroup per (unit, 8-row batch chunk), chunk partials in
 * `partials`, folded in a fixed order by a second launch (deterministic). context_dim <= 16. */
int encdiff_encoder_warp_fwd(const float* u, long ldu, int batch, int units, const float* params,
                             long unit_stride, int context_dim, float* out, long ldo, void* stream);
int encdiff_encoder_warp_bwd(const float* u, long ldu, int batch, int units, const float* params,
                             long unit_stride, int context_dim, const float* dout, long lddo, float* du,
                             long lddu, float* grads, float* partials, void* stream);
/* Encoder4's trunk head (openaimodel_enc.py:1012-1013): View((-1, d*16)) of the NCHW 4x4 trunk
 * output + Linear(d*16, units), read straight from the trunk's NHWC fp32 rows r [batch*16][ldr]
 * (element (b, c, p) at r[(b*16 + p)*ldr + c], column k = c*16 + p of W [units][d*16], the
 * reference layout).  fp32.  fwd: u [batch][ldu] = x W^T + bias.  bwd (one launch): dr (bf16
 * NHWC rows, the trunk's output gradient) = du W, dW += du^T x, db += sum_b du (batch order,
 * deterministic).  Replaces the flatten copy, the Linear GEMMs and their gradient adds. */
int encdiff_encoder_head_fwd(const float* r, long ldr, int batch, int d, const float* W, const float* bias,
                             int units, float* u, long ldu, void* stream);
int encdiff_encoder_head_bwd(const float* r, long ldr, int batch, int d, const float* W, int units,
                             const float* du, long lddu, void* dr, long lddr, float* dW, float* db,
                             void* stream);
/* fp32 scratch the backward needs for its per-batch-chunk weight-gradient partials. */
int encdiff_encoder_warp_partials_floats(int batch, int units, long unit_stride);

/* Encoder4 convolution trunk (openaimodel_enc.py:1002-1012, EncResBlock :969-989) runs on
 * encdiff_gemm (Conv2d(k4,s2,p1): RESAMPLE_K4S2 / K4S2_T im2col modes; 3x3 and 1x1 convs)
 * and these training-mode BatchNorm2d kernels over NHWC bf16 rows (nn.BatchNorm2d.train():
 * batch statistics over N*H*W, biased variance to normalise, running stats updated with
 * `momentum` and the unbiased variance).
 *   fwd: y = act((x - mean) * rstd * gamma + beta), act = ReLU if relu; writes mean/rstd.
 *   bwd: g = dy * act'(z) (z recomputed), dgamma += sum g*xhat, dbeta += sum g,
 *        dx = gamma*rstd*(g - mean(g) - xhat*mean(g*xhat)).
 * Each reduction is one launch whose last workgroup folds per-workgroup partials in a
 * fixed order (fp64): deterministic.  `partials` holds
 * encdiff_batchnorm_partials_floats(rows, c) floats; `counter` is a zero-initialised
 * device uint32 the kernels leave at zero.  c % 8 == 0, 256 % c == 0. */
typedef struct EncdiffBatchNormArgs {
  int rows, c;
  float eps, momentum;
  int relu, x_f32;                  /* x_f32: x is fp32 (else bf16)                  */
  const void* x; long ldx;          /* [rows][c] pre-BN activations, bf16 or fp32    */
  const float* gamma; const float* beta;
  void* y; long ldy;                /* fwd: bf16 out                                 */
  float* mean; float* rstd;         /* [c]: written by fwd, read by bwd              */
  float* running_mean; float* running_var;  /* optional (fwd)                        */
  float* partials;                  /* scratch                                       */
  unsigned int* counter;
  const void* dy; long lddy;        /* bwd: gradient of the (activated) output       */
  void* dx; long lddx;              /* bwd: bf16 out                                 */
  float* dgamma; float* dbeta;      /* bwd: fp32 +=                                  */
  int y_split, pad2_;               /* fwd / apply: y as split-bf16 blocks [hi|lo|hi] of c
                                       channels each (bf16x3 GEMM operand), else plain bf16 */
} EncdiffBatchNormArgs;

int encdiff_batchnorm_partials_floats(int rows, int c);
int encdiff_batchnorm_fwd(const EncdiffBatchNormArgs* args, void* stream);
int encdiff_batchnorm_bwd(const EncdiffBatchNormArgs* args, void* stream);
/* Eval-mode BatchNorm2d (+ReLU) (BatchNorm2d.eval(): running statistics): y = (x - mean) *
 * rstd * gamma + beta with the caller's mean / rstd; no reduction (validation encoding pass,
 * ddpm_enc.py:377-390).  partials / counter are not used. */
int encdiff_batchnorm_apply(const EncdiffBatchNormArgs* args, void* stream);

/* fp32 NCHW [batch][c][hw] -> bf16 rows [batch*hw][ldy], channels c..cpad-1 zero
 * (the image as the first Encoder4 conv's im2col source, channels padded to 8). */
int encdiff_nchw_to_rows(const float* x, int batch, int c, int hw, int cpad, void* y, long ldy, void* stream);
/* The same as split-bf16 blocks [hi | lo | hi] of cpad channels each (ldy >= 3 * cpad). */
int encdiff_nchw_to_rows_split3(const float* x, int batch, int c, int hw, int cpad, void* y, long ldy,
                                void* stream);

/* ---------------------------------------------------------------- SpatialTransformer tail
 * Everything of a SpatialTransformer after its self-attention is row-local (attention.py:211-215,
 * 250-261): t1 = to_out(o1) + t0; q2 = to_q(LN2(t1)); o2 = softmax(q2 k2^T * scale) v2 over the
 * image's concept tokens; t2 = to_out(o2) + t1; f = proj(LN3(t2)); a = f_v * gelu(f_g);
 * t3 = ff2(a) + t2; out = proj_out(t3) + x.  ONE kernel runs the chain for a tile of rows with
 * the rows resident in LDS (fp32 residual stream) and the weights streamed from L2, instead of
 * seven launches (GEMMs, cross-attention, LayerNorms).  Weights are the bf16 GEMM operands
 * [out][in] (row stride ld_*); biases / LayerNorm affine fp32.  The save_* pointers (all NULL or
 * all set) receive the activations the backward reads (training forward): t1, n2, q2, o2, t2,
 * n3, f, a, t3 (bf16 [rows][..]), s2 / s3 (fp32 [rows][2] mean, rstd), lse2 (fp32
 * [batch*heads][tokens], natural-log).  Supported: (c, heads) in {(64, 8), (128, 8), (256, 8)},
 * n_ctx <= 64, rows a multiple of the row tile (64; 32 at c = 256) and tile / tokens nested;
 * ENCDIFF_ERR_UNSUPPORTED / _SHAPE otherwise (the caller then issues the separate launches). */
typedef struct EncdiffStTailArgs {
  int rows, c, tokens, heads, n_ctx;
  float ln_eps, scale;
  int pad_;                     /* 0; timing experiments only (tools/st_tail_bench.py): stage mask */
  const void* o1; long ld_o1;   /* self-attention output      */
  const void* t0; long ld_t0;   /* proj_in output (residual)  */
  const void* x; long ld_x;     /* block input (residual of proj_out) */
  const void* k2; const void* v2; long ld_kv;  /* [batch*n_ctx][..] concept-token keys / values */
  const void* w_out1; long ld_out1; const float* b_out1;
  const float* g2; const float* be2;
  const void* w_q2; long ld_q2;
  const void* w_out2; long ld_out2; const float* b_out2;
  const float* g3; const float* be3;
  const void* w_ff1; long ld_ff1; const float* b_ff1;   /* [8c][c]: value rows, then gate rows */
  const void* w_ff2; long ld_ff2; const float* b_ff2;   /* [c][4c] */
  const void* w_po; long ld_po; const float* b_po;
  void* out; long ld_out;
  void* save_t1; void* save_n2; void* save_q2; void* save_o2; void* save_t2; void* save_n3;
  void* save_f; void* save_a; void* save_t3; long ld_save; /* ld of the [rows][c] saves (f: 8c, a: 4c dense) */
  float* save_s2; float* save_s3; float* save_lse2;
  float* gn_stats; long ld_gn_stats;  /* optional: the next GroupNorm's producer statistics of out
                                         (EncdiffGemmArgs.gn_stats layout; needs rows % 64 == 0) */
  int gn_stats_add;                   /* 1: gn_stats is zeroed by the caller and two 32-row tiles
                                         add their halves of a segment atomically (0 + a + b: the
                                         same bits in either order) -- twice the workgroups when a
                                         64-row tile would leave CUs idle; 0: written by one tile */
  int pad2_;
  void* head_t2; void* head_n3; long ld_head;  /* optional (inference, no saves): stop after norm3 --
                                         t2 and n3 = LN3(t2) written here (bf16 rows); the
                                         feed-forward and proj_out are the caller's launches (c = 256
                                         at sampling batches, where one workgroup streaming the
                                         feed-forward's 1.5 MB of weights is the slow part) */
} EncdiffStTailArgs;

int encdiff_st_tail_fwd(const EncdiffStTailArgs* args, void* stream);

/* The row-local head of a SpatialTransformer (attention.py:250-254, 211): gn = GroupNorm32(x)
 * (from the producer's segment sums gn_in_stats, EncdiffGemmArgs.gn_stats layout, when given --
 * then gn and the per-(image, group) mean / rstd gn_stats are written; with gn_in_stats == gn == NULL
 * the workgroup computes the statistics of its images from x itself and gn is not written
 * (inference); else gn is read, computed by encdiff_groupnorm_fwd), t0 = proj_in(gn),
 * n1 = LN1(t0), qkv = n1 [Wq; Wk; Wv]^T, as one kernel
 * (c in {64, 128}).  n1 / s1 optional (training saves).  Replaces up to three launches. */
typedef struct EncdiffStHeadArgs {
  int rows, c, tokens, pad_;
  float gn_eps, ln_eps;
  const void* x; long ld_x;
  const float* gn_in_stats; long ld_gn_in_stats;
  const float* gn_gamma; const float* gn_beta;
  void* gn; long ld_gn;
  float* gn_stats;                  /* [batch][32][2] (with gn_in_stats) */
  const void* w_in; long ld_in; const float* b_in;
  const float* g1; const float* be1;
  const void* w_qkv; long ld_w_qkv; /* [3c][c] */
  void* t0; long ld_t0;
  void* n1; long ld_n1;
  float* s1;                        /* [rows][2] mean, rstd */
  void* qkv; long ld_qkv;
} EncdiffStHeadArgs;

int encdiff_st_head_fwd(const EncdiffStHeadArgs* args, void* stream);

/* Backward of the row-local tail of a SpatialTransformer (attention.py:211-215 BasicTransformerBlock
 * after attn1, :226-232 GEGLU, :170-191 CrossAttention to the concept tokens, :260-261 proj_out)
 * as ONE kernel: the input-gradient chain of encdiff_st_tail_fwd for a tile of token rows, with
 * the rows resident in LDS (fp32 residual-gradient stream, bf16 MFMA operands):
 *   d_t3 = dy Wpo;  d_a = d_t3 W2;  d_f = GEGLU'(f) (d_a);  d_n3 = d_f W1
 *   d_t2 = d_t3 + LN3'(t2; d_n3);   d_o2 = d_t2 Wout2
 *   (d_q2, dK2, dV2) = cross-attention backward (recomputed from q2, K2 / V2, the saved LSE)
 *   d_n2 = d_q2 Wq2;  d_t1 = d_t2 + LN2'(t1; d_n2);  d_o1 = d_t1 Wout1
 * It writes the gradients the weight-gradient GEMMs and the self-attention backward read
 * (d_t3 d_f d_t2 d_q2 d_t1 d_o1), the LN2 / LN3 affine partial sums of the tile (row blockIdx of
 * the part matrices) and dK2 / dV2 of the image's concept tokens (a tile per image: written;
 * several: fp32 partial slabs combined in tile order by the image's last tile through a ticket
 * -- reproducible).  Weights are the TRANSPOSED bf16 copies ([in][out] of each Linear, dense).
 * Replaces 9 launches of the unfused backward (6 input-gradient GEMMs with their weight-gradient
 * pairs, two LayerNorm backwards, the cross-attention backward); the weight gradients are the
 * caller's (one grouped launch).  c in {64, 128}, heads == 8, n_ctx <= 64, tokens a multiple of
 * the row tile (64; 32 at c = 128 with fewer than 256 64-row tiles).  Reference of the chain:
 * attention.py:180-191 (attention), :206-215 (block), :226-232 (GEGLU), :250-261 (transformer). */
typedef struct EncdiffStTailBwdArgs {
  int rows, c, tokens, heads, n_ctx;
  float scale;                               /* dh^-0.5 */
  int part_rows;                             /* rows of the LN partial matrices (>= launched tiles) */
  int pad_;                                  /* 0; timing experiments only (tools/st_bwd_bench.py): stage mask */
  const void* dy; long ld_dy;                /* d(block output), bf16 [rows][c] */
  const void* f; long ld_f;                  /* saved GEGLU input [rows][8c]: value | gate */
  const void* t2; const void* t1; const void* q2; const void* o2; long ld_save;
  const float* s3; const float* s2;          /* saved LN3 / LN2 (mean, rstd) [rows][2] */
  const float* lse2;                         /* saved cross-attention LSE [batch*heads][tokens] */
  const void* k2; const void* v2; long ld_kv;  /* [batch*n_ctx][..] concept-token keys / values */
  const void* w_po_t;                        /* [c][c]   proj_out^T        */
  const void* w_ff2_t;                       /* [4c][c]  ff.net.2^T        */
  const void* w_ff1_t;                       /* [c][8c]  ff.net.0.proj^T   */
  const void* w_out2_t;                      /* [c][c]   attn2.to_out^T    */
  const void* w_q2_t;                        /* [c][c]   attn2.to_q^T      */
  const void* w_out1_t;                      /* [c][c]   attn1.to_out^T    */
  const float* g3; const float* g2;          /* LN3 / LN2 gamma            */
  void* d_t3; void* d_t2; void* d_q2; void* d_t1; void* d_o1; long ld_d;  /* bf16 [rows][c] outputs */
  void* d_f; long ld_df;                     /* bf16 [rows][8c]            */
  float* ln3_dg; float* ln3_db; float* ln2_dg; float* ln2_db; long ld_part;
  void* dk2; void* dv2; long ld_dkv;         /* bf16 [batch*n_ctx][..]: written when a tile holds a
                                                whole image (tokens == tile rows) */
  float* kv_part;                            /* tokens > tile: fp32 [rows/tile][n_ctx][2c] partial slabs
                                                of dK2 | dV2 per tile, folded into dk2 / dv2 by
                                                encdiff_st_head_bwd (kv_* fields) */
} EncdiffStTailBwdArgs;

int encdiff_st_tail_bwd(const EncdiffStTailBwdArgs* args, void* stream);
/* The row tile encdiff_st_tail_bwd uses for (c, rows, tokens): tokens / tile partial slabs per image. */
int encdiff_st_tail_bwd_tile(int c, int rows, int tokens);

/* Backward of the row-local head (attention.py:211 norm1 + attn1's q/k/v, :253-254 proj_in) after
 * the self-attention backward, as ONE kernel for a tile of token rows:
 *   d_n1 = d_qkv [Wq; Wk; Wv];  d_t0 = d_t1 + LN1'(t0; d_n1);  d_gn = d_t0 Win
 * writing d_t0 (proj_in's weight gradient reads it), d_gn (the GroupNorm backward reads it) and
 * the LN1 affine partial sums (row blockIdx).  Weights transposed ([in][out], dense).  c in {64, 128}.
 * kv_part (optional): the tail kernel's dK2 / dV2 partial slabs, kv_tiles per image, summed in tile
 * order into dk2 / dv2 (bf16) by the same grid (no ticket, reproducible). */
typedef struct EncdiffStHeadBwdArgs {
  int rows, c, part_rows, pad_;
  const void* d_qkv; long ld_dqkv;           /* bf16 [rows][3c] */
  const void* d_t1; long ld_dt1;             /* residual gradient, bf16 [rows][c] */
  const void* t0; long ld_t0; const float* s1;
  const float* g1;
  const void* w_qkv_t;                       /* [c][3c] */
  const void* w_in_t;                        /* [c][c]  */
  void* d_t0; long ld_dt0;
  void* d_gn; long ld_dgn;
  float* ln1_dg; float* ln1_db; long ld_part;
  const float* kv_part; int kv_tiles, n_ctx, batch, pad2_;
  void* dk2; void* dv2; long ld_dkv;
} EncdiffStHeadBwdArgs;

int encdiff_st_head_bwd(const EncdiffStHeadBwdArgs* args, void* stream);

/* The weight gradients of a fused transformer block's Linear layers (attention.py:160-167, 206-215,
 * 226-232, 253-261: proj_out, ff.net.2, ff.net.0.proj, attn2.to_out / to_q, attn1.to_out, to_q/k/v,
 * proj_in): dW_i += dY_i^T X_i and db_i += column sums of dY_i over the K tokens, for up to 16 problems
 * in ONE grid (+ a fold launch when a block is split over token chunks: fp32 slabs in the caller's
 * workspace summed in chunk order -- reproducible).  M, N multiples of 64, K of 32; operands bf16,
 * 16-byte aligned.  plan (host, no device access) writes the launch description into `blob` (NULL:
 * only *blob_bytes); the caller copies it to device memory once and launches it any number of times
 * (captured graphs: the blob and the slab region must outlive them). */
typedef struct EncdiffWgradProb {
  const void* dy; long ld_dy;     /* bf16 [K][M] */
  const void* x; long ld_x;       /* bf16 [K][N] */
  float* dw; long ld_dw;          /* fp32 [M][N], accumulated */
  float* db;                      /* fp32 [M], accumulated (optional) */
  int M, N, K, pad_;
} EncdiffWgradProb;

int encdiff_st_wgrad_plan(const EncdiffWgradProb* probs, int n, float* workspace, long ws_floats, void* blob,
                          long capacity, long* blob_bytes);
int encdiff_st_wgrad_launch(const void* host_blob, const void* dev_blob, void* stream);
/* the weight-gradient grid alone (no fold): the caller hands the plan's fold to the next GroupNorm
   backward (EncdiffGroupNormArgs.fold_plan = dev_blob, fold_blocks = *fold_blocks) */
int encdiff_st_wgrad_launch_nofold(const void* host_blob, const void* dev_blob, void* stream, const void** fold_plan,
                                   int* fold_blocks);

/* ---------------------------------------------------------------- step prologue
 * The per-step device work in front of the training step, as ONE launch:
 *   - zero jobs: 2-D byte regions set to 0 (the gradient arena, producer-statistics slots that
 *     the step's kernels add into); ptr and row_bytes / ld_bytes multiples of 16;
 *   - t[b] ~ U{0 .. timesteps-1} (LatentDiffusion.forward, ddpm_enc.py:1041) and noise[i] ~ N(0, 1)
 *     (p_losses, ddpm_enc.py:1184 torch.randn_like(x_start)), Philox4x32-10 keyed by `seed`
 *     with the device counter *rng_counter (stream offsets: noise element i uses block i / 4 of
 *     stream 0, t[b] block b of stream 1), then Box-Muller on uniforms in (0, 1];
 *   - *rng_counter += 1 and, when given, *data_step += 1 (the image pool's epoch step read by
 *     encdiff_gather_images_u8 earlier in the step) by the last workgroup to finish (ticket
 *     `done`, zero on entry, left zero), so a captured step advances both by itself.
 * t or noise may be NULL (a test feeding its own). */
/* One convolution of an inference ResBlock with the GroupNorm in front of it, as ONE launch
 * (openaimodel_enc.py:255-275 with use_scale_shift_norm, replacing the GroupNorm launch, the conv
 * launch and -- for conv2 -- the skip / resample launch of the unfused path):
 *   y = conv3x3(resample(SiLU(GN(x) (1 + scale) + shift))) + bias + skip
 * A workgroup stages the whole images its output rows read into LDS, reduces their GroupNorm
 * statistics, normalises them in place (bf16, as the GroupNorm launch would store them), applies
 * the 2x resample (DOWN2: avg-pool of the normalised rows, rounded to bf16 as the resample pass
 * stores it; UP2: nearest, read through the gather), and runs the implicit-im2col GEMM of its
 * 16-row tiles x 16-column slice on MFMA with the weights streamed from L2.  skip: resid (bf16 rows
 * at the output resolution, or read through resid_resample from the ResBlock input) or a 1x1
 * skip conv (out += bf16(xskip Wskip^T + bskip), as the skip launch would store it).
 * Constraints: cin % 32 == 0, cout % 16 == 0, square images, the staged images fit in LDS
 * (ENCDIFF_ERR_UNSUPPORTED otherwise: the caller issues the unfused launches). */
typedef struct EncdiffResConvArgs {
  int batch, h, cin, cout;       /* x: batch images of h x h pixels, cin channels             */
  int resample;                  /* ENCDIFF_RESAMPLE_*: after the GroupNorm (conv at 2h / h/2) */
  int groups, silu;
  float eps;
  const void* x; long ld_x;      /* bf16 rows [batch*h*h][cin]                                 */
  const float* gamma; const float* beta;
  const float* film; long ld_film;  /* optional fp32 [batch][ld_film]: scale at [c], shift at
                                       [cin + c]; ld_film 0: one row for every image          */
  const void* w; long ld_w;      /* bf16 [cout][9*cin] (tap-major, channels-last)              */
  const float* bias;             /* optional fp32 [cout]                                       */
  const void* resid; long ld_resid;  /* optional bf16 rows added to the output               */
  int resid_resample;            /* resid at the output resolution (NONE), its half (UP2: nearest)
                                    or its double (DOWN2: 2x2 average rounded to bf16)        */
  int cskip;                     /* 1x1 skip conv input channels (0: none)                     */
  const void* xskip; long ld_xskip;  /* bf16 rows [batch*ho*ho][cskip]                        */
  const void* wskip; long ld_wskip;  /* bf16 [cout][cskip]                                    */
  const float* bskip;            /* optional fp32 [cout]                                       */
  void* y; long ld_y;            /* bf16 rows [batch*ho*ho][cout]                              */
  int tile_m, tile_n;            /* plan overrides (0: heuristic): 16-row tiles per workgroup
                                    (1, 2, 4), 16-column tiles per workgroup (1, 2)           */
  int skip_stages;               /* 0; timing experiments only (tools/rc_bench.py): 1 no staging
                                    loads, 2 no normalisation, 4 no GEMM (nor its B staging), 8 no
                                    stores, 16 no B staging, 32 no GEMM arithmetic, 64 kl = 0,
                                    128 return at entry, 256 return once every operand landed */
  int pad_;
} EncdiffResConvArgs;

int encdiff_resconv_fwd(const EncdiffResConvArgs* args, void* stream);
/* The plan of encdiff_resconv_fwd for these arguments without launching (pointers are not read):
 * ENCDIFF_OK and the LDS bytes / workgroups per launch, or the error the launch would return. */
int encdiff_resconv_query(const EncdiffResConvArgs* args, int* lds_bytes, int* grid);

typedef struct EncdiffZeroJob {
  void* ptr;
  long long rows, row_bytes, ld_bytes;
} EncdiffZeroJob;

typedef struct EncdiffStepPrologueArgs {
  const EncdiffZeroJob* jobs;  /* device array */
  int njobs;
  int batch;
  int timesteps;
  int pad_;
  unsigned long long seed;
  long long* rng_counter;      /* device */
  long long* data_step;        /* device, optional */
  long long* t;                /* device int64 [batch], optional */
  float* noise;                /* device fp32 [n_noise], optional */
  long long n_noise;
  int* done;                   /* device ticket */
  int pad2_;
} EncdiffStepPrologueArgs;

int encdiff_step_prologue(const EncdiffStepPrologueArgs* args, void* stream);

/* Library/device information (for tests): returns the number of exported kernels. */
int encdiff_version(void);

#ifdef __cplusplus
}
#endif
#endif /* ENCDIFF_HIP_H */
