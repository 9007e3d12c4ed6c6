/*
 * ska_sdp_hip.h -- C ABI of the MI355X-native predict/invert + calibration
 * hot path (libska_sdp_hip.so, hand-written HIP for gfx950).
 *
 * Every entry point takes DEVICE pointers (plain pointers + sizes + strides,
 * no torch types), an optional hipStream_t passed as void*, and an error
 * buffer.  It returns SDP_HIP_OK or one of the error codes below, which the
 * Python layer maps back onto the reference's exception types
 * (AssertionError / ValueError / RuntimeError).
 *
 * Outputs are always caller-allocated (the ska-sdp-func convention of
 * dft_point_v00, reference src/ska_sdp_func_python/imaging/dft.py:169-178);
 * the library never returns memory it allocated.  Internal scratch
 * (visibility records, w-plane grids, FFT plans) lives in a per-device cache
 * that grows on demand and is released by sdp_hip_release_workspace().
 */
#ifndef SKA_SDP_HIP_H
#define SKA_SDP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define SDP_HIP_OK 0
#define SDP_HIP_ERR_INVALID_ARG 1 /* -> ValueError   */
#define SDP_HIP_ERR_RUNTIME 2     /* -> RuntimeError */
#define SDP_HIP_ERR_NO_DEVICE 3   /* -> RuntimeError */
#define SDP_HIP_ERR_MEMORY 4      /* -> MemoryError  */

/* ---- dtype codes ------------------------------------------------------- */
#define SDP_HIP_F32 1
#define SDP_HIP_F64 2
#define SDP_HIP_C64 3
#define SDP_HIP_C128 4

/* ---- flags for the NUFFT pair ------------------------------------------ */
#define SDP_HIP_FLIP_UW 1u    /* negate u and w on the fly (RASCIL, ng.py:210-213) */
#define SDP_HIP_ACCUMULATE 2u /* add into the output instead of overwriting      */
#define SDP_HIP_BATCH_FIRST 4u /* sdp_hip_ms2dirty_batch: first batch (zero the planes) */
#define SDP_HIP_BATCH_LAST 8u  /* sdp_hip_ms2dirty_batch: last batch (FFT + screens)    */
/* sdp_hip_ms2dirty / _vis: bucket every in-grid visibility (zero weights too,
 * they add exact zeros; info.nvis_used then counts them) and keep the
 * bucketing on the device for following SDP_HIP_REUSE_BUCKETS calls */
#define SDP_HIP_KEEP_BUCKETS 16u
/* sdp_hip_ms2dirty / _vis: reuse the kept bucketing (invert_ng's other
 * polarisations): the same uvw and freq arrays, unchanged, and the same nrow,
 * nchan, image geometry, epsilon, do_wstacking and FLIP_UW as the keeping
 * call; only the visibilities, weights, flags and pol differ.  Only the value
 * pass, gridding and FFT run.  Any other wstack call (or a workspace release)
 * in between drops the kept bucketing: the call then fails with
 * SDP_HIP_ERR_INVALID_ARG. */
#define SDP_HIP_REUSE_BUCKETS 32u
/* epsilon below 1e-7 (the reference's default 1e-12 included) runs the fp64
 * NUFFT: W = ceil(-log10(epsilon/10)) in [9, 16], fp64 taps, records, c128
 * planes, Z2Z FFTs, one-cell buckets (grids whose (first plane, cell)
 * histogram exceeds 2^28 keys are refused).  SDP_HIP_FP32 keeps the fp32
 * NUFFT at its floor instead (W = 8, ~1e-6 relative RMS), as before. */
#define SDP_HIP_FP32 64u
/* sdp_hip_ms2dirty_batch: grid one w slab of the sequence's plane layout.
 * `bounds` then holds 8 doubles: the 6 below, then the slab's first planes
 * [lo, hi) (integers, 0 <= lo < hi; hi is clipped to the layout's first-plane
 * count, which sdp_hip_wstack_layout reports).  Only visibilities whose first
 * w plane lies in the slab are gridded -- the others are skipped (tested
 * before their weights or values are read) -- and only planes lo .. hi + W - 2
 * are held, transformed and screened.  The dirty images of the slabs of one
 * layout sum to the full image (multi-GPU w-slab partition).
 * fp32 NUFFT (epsilon >= 1e-7 or SDP_HIP_FP32) with w-stacking only. */
#define SDP_HIP_W_SLAB 128u
/* sdp_hip_ms2dirty / _vis / sdp_hip_dirty2ms / _vis: use the second set of
 * scratch buffers (planes, records, histograms, FFT plans, auxiliary stream).
 * A caller that alternates it between two streams can have two calls in
 * flight at once -- the next call's bucketing runs while the previous one
 * grids and transforms.  Not with KEEP/REUSE_BUCKETS, the batch flags or
 * W_SLAB. */
#define SDP_HIP_SLOT1 256u

/* Diagnostics filled by the NUFFT entry points (may be NULL). */
typedef struct sdp_hip_wgrid_info {
    int support;          /* ES kernel support W                            */
    double beta;          /* ES kernel shape                                */
    int ngrid_x, ngrid_y; /* oversampled grid (sigma = 2)                   */
    int nplanes;          /* w planes (1 when do_wstacking == 0)            */
    double w0, dw;        /* plane 0 position and spacing (wavelengths)     */
    int64_t nvis_used;    /* visibilities with non-zero weight              */
    int64_t nitems;       /* gridding work items launched                   */
    int plane_chunk;      /* planes resident per pass                       */
    float ms_prep, ms_grid, ms_fft, ms_screen; /* stage times if timing on  */
    int bucket;           /* bucket edge in cells: 1 = one-cell buckets,
                             16 = 16x16-cell buckets sub-sorted by cell
                             (large grids)                                  */
    int grid_launches;    /* (de)gridding kernel launches (one per plane
                             chunk); ms_grid is their summed time           */
    int padded;           /* invert: gridded on cells padded to 4 records
                             (k_grid_mfma_pad; 0: k_grid_mfma)              */
    int fp64;             /* the fp64 NUFFT ran (epsilon < 1e-7)            */
    int tiled;            /* one-cell buckets from the two-level (64x64-cell
                             bin, then cell) LDS-histogram sort             */
} sdp_hip_wgrid_info;

/* Library/ABI version and a device probe. */
int sdp_hip_version(void);
int sdp_hip_device_count(int *count, char *errbuf, size_t errbuf_len);
int sdp_hip_release_workspace(char *errbuf, size_t errbuf_len);
/* When non-zero, the NUFFT entry points time their stages with HIP events
 * (adds stream synchronisations; off by default). */
int sdp_hip_set_stage_timing(int enable);

/*
 * sdp_hip_ms2dirty -- replaces ducc0.wgridder.ms2dirty as called by
 * invert_ng (reference src/ska_sdp_func_python/imaging/ng.py:240-256 MFS,
 * :271-287 per channel; double_precision_accumulation=True).
 *
 * dirty[x,y] = sum_{row,chan} wgt * Re{vis * exp(2 pi i (u l_x + v m_y - w (n-1)))} [/n]
 * (ducc0 convention, l_x = (x - nx/2) pixsize_x).
 *
 * uvw      [nrow, 3] f64 metres, row stride uvw_row_stride (elements)
 * freq     [nchan] f64 Hz
 * vis      [nrow, nchan] c64 or c128 (vis_dtype SDP_HIP_C64 / SDP_HIP_C128)
 *          with element strides; NULL means unit visibilities (PSF,
 *          ng.py:231-233)
 * wgt      [nrow, nchan] f32 or f64 (wgt_dtype SDP_HIP_F32 / SDP_HIP_F64; ducc0
 *          takes f64) with element strides; NULL means unit weights.  Samples
 *          of zero weight are skipped (their visibilities are never read)
 * dirty    f64, element (x, y) at dirty[x*dirty_stride_x + y*dirty_stride_y]
 *          (pass strides (1, nx) to receive RASCIL's transposed image)
 * epsilon  requested accuracy: >= 1e-7 the fp32 NUFFT (W = ceil(-log10(eps/10)),
 *          <= 8); below 1e-7 the fp64 NUFFT (W in [9, 16], c128 planes) unless
 *          flags has SDP_HIP_FP32 (fp32 at its floor, W = 8)
 */
int sdp_hip_ms2dirty(const double *uvw, int64_t uvw_row_stride,
                     const double *freq, int nchan, int64_t nrow,
                     const void *vis, int vis_dtype, int64_t vis_row_stride,
                     int64_t vis_chan_stride, const void *wgt, int wgt_dtype,
                     int64_t wgt_row_stride, int64_t wgt_chan_stride,
                     int npix_x, int npix_y, double pixsize_x,
                     double pixsize_y, double epsilon, int do_wstacking,
                     unsigned flags, double *dirty, int64_t dirty_stride_x,
                     int64_t dirty_stride_y, void *stream,
                     sdp_hip_wgrid_info *info, char *errbuf,
                     size_t errbuf_len);

/*
 * sdp_hip_ms2dirty_batch -- sdp_hip_ms2dirty over a sequence of visibility
 * batches that share one w-plane layout and one set of resident uv planes
 * (a band too large for one call, e.g. the 13.4 Gvis of C4 on fewer than 8
 * GPUs, streamed through the device channel block by channel block).  Every
 * call of a sequence passes the same image geometry, epsilon, do_wstacking,
 * FLIP_UW and `bounds`; the first carries SDP_HIP_BATCH_FIRST (planes
 * zeroed), the last SDP_HIP_BATCH_LAST (FFT, w-screens, grid correction into
 * `dirty`, which may be NULL before).  The result equals one sdp_hip_ms2dirty
 * call over all batches with that plane layout.
 * bounds   host {min w, max w, max|u|, max|v|} over ALL batches in metres
 *          (uvw as given, before FLIP_UW) and {min freq, max freq} over all
 *          batches' frequencies (6 doubles)
 * Replaces the reference's per-(pol, chan) ducc0 loop as a streaming form of
 * ms2dirty (ng.py:259-289); the planes must all fit on the device.  A batch
 * whose visibilities fall outside `bounds` fails with SDP_HIP_ERR_INVALID_ARG,
 * and so does a later batch when its sequence's planes are gone (another
 * NUFFT call or a workspace release after the first batch) or its geometry,
 * epsilon, flags or bounds differ from the first batch's.
 */
int sdp_hip_ms2dirty_batch(const double *uvw, int64_t uvw_row_stride,
                           const double *freq, int nchan, int64_t nrow,
                           const void *vis, int vis_dtype,
                           int64_t vis_row_stride, int64_t vis_chan_stride,
                           const void *wgt, int wgt_dtype, int64_t wgt_row_stride,
                           int64_t wgt_chan_stride, int npix_x, int npix_y,
                           double pixsize_x, double pixsize_y, double epsilon,
                           int do_wstacking, unsigned flags,
                           const double *bounds, double *dirty,
                           int64_t dirty_stride_x, int64_t dirty_stride_y,
                           void *stream, sdp_hip_wgrid_info *info,
                           char *errbuf, size_t errbuf_len);

/*
 * sdp_hip_wstack_layout -- the w-plane layout sdp_hip_ms2dirty_batch uses for
 * `bounds` (6 doubles, as above) and the image geometry, without device work:
 * info->support, nplanes (first planes = nplanes - support + 1), w0, dw,
 * ngrid_x/y, fp64.  A w-slab partition (SDP_HIP_W_SLAB) splits the first
 * planes [0, nplanes - support + 1) between the ranks.
 */
int sdp_hip_wstack_layout(const double *bounds, int npix_x, int npix_y,
                          double pixsize_x, double pixsize_y, double epsilon,
                          int do_wstacking, unsigned flags, sdp_hip_wgrid_info *info,
                          char *errbuf, size_t errbuf_len);

/*
 * sdp_hip_ms2dirty_vis -- sdp_hip_ms2dirty with the visibility-side prologue
 * of invert_ng fused into its first pass, so the
 * Visibility's own arrays are read in place:
 *   flagged_vis / flagged_imaging_weight (reference imaging/ng.py:191, :202;
 *   value * (1 - flags)), convert_pol_frame (ng.py:193-198) and the weight sum
 *   sumwt (ng.py:258, :289).
 * vis       [nrow, nchan, npol_vis] c64/c128 at pol 0, element strides
 *           (row, chan, pol); NULL = unit visibilities (PSF)
 * pol_coeff host array of 2*npol_vis doubles (re, im): image-pol visibility =
 *           sum_k coeff_k * vis_k * (1 - flag_k) (one row of the conversion
 *           matrix); NULL = no conversion, the image pol is vis pol `pol`
 * wgt       weights of image pol `pol` (f32 or f64, wgt_dtype), strides
 *           (row, chan); NULL = ones
 * vis_flags [nrow, nchan, npol_vis] integers of flag_bytes at pol 0 with
 *           strides, or NULL; the weight is masked with flag pol `pol`
 * sumwt     device double, += sum over rows and channels of the masked
 *           weights (NULL: not computed)
 * shift_lmn host array (l, m, n-1) of the image phase centre relative to the
 *           visibility phase centre, or NULL: shift_vis_to_image's tangent
 *           phase rotation (reference imaging/base.py:48-92,
 *           visibility/base.py:27-90) applied on the fly, vis *
 *           exp(+2 pi i uvw_lambda . lmn) (uvw as given, before FLIP_UW)
 * Other arguments as sdp_hip_ms2dirty.
 */
int sdp_hip_ms2dirty_vis(const double *uvw, int64_t uvw_row_stride,
                         const double *freq, int nchan, int64_t nrow,
                         const void *vis, int vis_dtype, int64_t vis_row_stride,
                         int64_t vis_chan_stride, int64_t vis_pol_stride,
                         int npol_vis, const double *pol_coeff, const void *wgt,
                         int wgt_dtype, int64_t wgt_row_stride,
                         int64_t wgt_chan_stride, const void *vis_flags,
                         int flag_bytes, int64_t flag_row_stride,
                         int64_t flag_chan_stride, int64_t flag_pol_stride,
                         int pol, int npix_x, int npix_y, double pixsize_x,
                         double pixsize_y, double epsilon, int do_wstacking,
                         unsigned flags, double *dirty, int64_t dirty_stride_x,
                         int64_t dirty_stride_y, double *sumwt,
                         const double *shift_lmn, void *stream,
                         sdp_hip_wgrid_info *info, char *errbuf,
                         size_t errbuf_len);

/*
 * sdp_hip_ms2dirty_vis_batch -- sdp_hip_ms2dirty_vis as one batch of a
 * sequence (SDP_HIP_BATCH_FIRST / _LAST in `flags`, `bounds` as
 * sdp_hip_ms2dirty_batch): invert_ng grids an MFS image's (or a cube
 * channel's) visibilities in channel batches through one set of resident w
 * planes when they are too many for one call (reference imaging/ng.py:
 * 240-256, one ducc0 call over all channels).  sumwt accumulates over the
 * batches.  Other arguments as sdp_hip_ms2dirty_vis.
 */
int sdp_hip_ms2dirty_vis_batch(const double *uvw, int64_t uvw_row_stride,
                               const double *freq, int nchan, int64_t nrow,
                               const void *vis, int vis_dtype, int64_t vis_row_stride,
                               int64_t vis_chan_stride, int64_t vis_pol_stride,
                               int npol_vis, const double *pol_coeff, const void *wgt,
                               int wgt_dtype, int64_t wgt_row_stride,
                               int64_t wgt_chan_stride, const void *vis_flags,
                               int flag_bytes, int64_t flag_row_stride,
                               int64_t flag_chan_stride, int64_t flag_pol_stride,
                               int pol, int npix_x, int npix_y, double pixsize_x,
                               double pixsize_y, double epsilon, int do_wstacking,
                               unsigned flags, const double *bounds, double *dirty,
                               int64_t dirty_stride_x, int64_t dirty_stride_y,
                               double *sumwt, const double *shift_lmn, void *stream,
                               sdp_hip_wgrid_info *info, char *errbuf,
                               size_t errbuf_len);

/*
 * sdp_hip_ms2dirty_vis_pols -- every image pol of one invert_ng image channel
 * in one call (reference imaging/ng.py:240-289: one ducc0 ms2dirty per image
 * pol over the same uvw).  The pols share one bucketing, and one value pass
 * reads each visibility's pols, flags and weights once and writes every
 * pol's records; then each pol is gridded, transformed and screened into its
 * own image.  Results as npol_img sdp_hip_ms2dirty_vis calls, pol q with row
 * q of the conversion matrix, the weights and flag mask of pol q.
 * pol_coeff host array of 2*npol_img*npol_vis doubles: row q, vis pol k at
 *           2*(q*npol_vis+k) (re, im); NULL = identity (image pol q = vis pol q)
 * wgt       weights [nrow, nchan, >= npol_img] (f32 or f64), strides (row,
 *           chan, pol); required
 * dirty     image pol q at dirty + q*dirty_stride_pol, strides (x, y)
 * sumwt     device doubles, pol q at sumwt + q*sumwt_stride (+= its masked
 *           weight sum), or NULL
 * npol_img  1..npol_vis.  flags may not hold KEEP / REUSE / BATCH bits.
 * fp64 plans (epsilon < 1e-7 without SDP_HIP_FP32) and plans outside the
 * one-cell single-level bucketing run the pols as separate calls.
 * Other arguments as sdp_hip_ms2dirty_vis.
 */
int sdp_hip_ms2dirty_vis_pols(const double *uvw, int64_t uvw_row_stride,
                              const double *freq, int nchan, int64_t nrow,
                              const void *vis, int vis_dtype, int64_t vis_row_stride,
                              int64_t vis_chan_stride, int64_t vis_pol_stride,
                              int npol_vis, const double *pol_coeff, int npol_img,
                              const void *wgt, int wgt_dtype, int64_t wgt_row_stride,
                              int64_t wgt_chan_stride, int64_t wgt_pol_stride,
                              const void *vis_flags, int flag_bytes,
                              int64_t flag_row_stride, int64_t flag_chan_stride,
                              int64_t flag_pol_stride, int npix_x, int npix_y,
                              double pixsize_x, double pixsize_y, double epsilon,
                              int do_wstacking, unsigned flags, double *dirty,
                              int64_t dirty_stride_x, int64_t dirty_stride_y,
                              int64_t dirty_stride_pol, double *sumwt,
                              int64_t sumwt_stride, const double *shift_lmn,
                              void *stream, sdp_hip_wgrid_info *info, char *errbuf,
                              size_t errbuf_len);

/*
 * sdp_hip_dirty2ms -- replaces ducc0.wgridder.dirty2ms as called by
 * predict_ng (reference src/ska_sdp_func_python/imaging/ng.py:99-112 MFS,
 * :117-129 per channel).  Exact adjoint of sdp_hip_ms2dirty:
 * vis = wgt * sum_{x,y} dirty[x,y] exp(-2 pi i (u l_x + v m_y - w (n-1))) [/n]
 */
int sdp_hip_dirty2ms(const double *uvw, int64_t uvw_row_stride,
                     const double *freq, int nchan, int64_t nrow,
                     const double *dirty, int64_t dirty_stride_x,
                     int64_t dirty_stride_y, int npix_x, int npix_y,
                     double pixsize_x, double pixsize_y, const void *wgt,
                     int wgt_dtype, int64_t wgt_row_stride, int64_t wgt_chan_stride,
                     double epsilon, int do_wstacking, unsigned flags,
                     void *vis, int vis_dtype, int64_t vis_row_stride,
                     int64_t vis_chan_stride, void *stream,
                     sdp_hip_wgrid_info *info, char *errbuf,
                     size_t errbuf_len);

/*
 * sdp_hip_dirty2ms_vis -- sdp_hip_dirty2ms for ONE image pol of predict_ng
 * with the image -> visibility pol-frame conversion (reference
 * imaging/ng.py:131-136) fused into the write-back: every output pol k of
 * vis [nrow, nchan, npol_vis] (element strides row, chan, pol; vis points at
 * pol 0) receives coeff_k * (this pol's predicted visibility), coeff_k =
 * column `pol` of the conversion matrix, host array of 2*npol_vis doubles
 * (NULL: output pol 0 only).  Without SDP_HIP_ACCUMULATE all npol_vis pols
 * are overwritten (zero where nothing is predicted); call the first image pol
 * without and the others with SDP_HIP_ACCUMULATE.  No weights (predict_ng
 * passes none, ng.py:99-129).  shift_lmn (host (l, m, n-1) or NULL) applies
 * shift_vis_to_image(inverse=True): vis * exp(-2 pi i uvw_lambda . lmn).
 */
int sdp_hip_dirty2ms_vis(const double *uvw, int64_t uvw_row_stride,
                         const double *freq, int nchan, int64_t nrow,
                         const double *dirty, int64_t dirty_stride_x,
                         int64_t dirty_stride_y, int npix_x, int npix_y,
                         double pixsize_x, double pixsize_y, double epsilon,
                         int do_wstacking, unsigned flags, void *vis,
                         int vis_dtype, int64_t vis_row_stride,
                         int64_t vis_chan_stride, int64_t vis_pol_stride,
                         int npol_vis, const double *pol_coeff,
                         const double *shift_lmn, void *stream,
                         sdp_hip_wgrid_info *info, char *errbuf,
                         size_t errbuf_len);

/*
 * sdp_hip_dirty2ms_vis_pols -- every image pol of one predict_ng MFS call in
 * one call (reference imaging/ng.py:99-112 per image pol, :131-136 the pol
 * conversion): the pols share one bucketing; each image pol's planes are
 * built and degridded, and one write-back combines all pols into every
 * visibility pol.  Results as npol_img sdp_hip_dirty2ms_vis calls, the first
 * without and the others with SDP_HIP_ACCUMULATE, pol q with column q of the
 * conversion matrix.
 * dirty     image pol q at dirty + q*dirty_stride_pol, strides (x, y)
 * pol_coeff host array of 2*npol_img*npol_vis doubles: image pol q, vis pol k
 *           at 2*(q*npol_vis+k) (re, im); NULL = identity
 * Other arguments as sdp_hip_dirty2ms_vis.
 */
int sdp_hip_dirty2ms_vis_pols(const double *uvw, int64_t uvw_row_stride,
                              const double *freq, int nchan, int64_t nrow,
                              const double *dirty, int64_t dirty_stride_x,
                              int64_t dirty_stride_y, int64_t dirty_stride_pol,
                              int npol_img, int npix_x, int npix_y, double pixsize_x,
                              double pixsize_y, double epsilon, int do_wstacking,
                              unsigned flags, void *vis, int vis_dtype,
                              int64_t vis_row_stride, int64_t vis_chan_stride,
                              int64_t vis_pol_stride, int npol_vis,
                              const double *pol_coeff, const double *shift_lmn,
                              void *stream, sdp_hip_wgrid_info *info, char *errbuf,
                              size_t errbuf_len);

/*
 * sdp_hip_dft_point_v00 -- replaces ska_sdp_func.visibility.dft_point_v00
 * (reference src/ska_sdp_func_python/imaging/dft.py:173-178) and the cupy
 * dft_kernel (:185-262, :288-337).  Caller-allocated output, replaced (not
 * accumulated), all arrays C-contiguous:
 *   direction_cosines [ncomp, 3] f64 (l, m, n-1)
 *   fluxes            [ncomp, flux_nchan, npol] c128; flux_nchan == nchan
 *                     or 1 (broadcast over channels, as numpy does in
 *                     dft_cpu_looped, dft.py:284)
 *   uvw_lambda        [ntimes*nbaselines, nchan, 3] f64 wavelengths
 *   vis               [ntimes*nbaselines, nchan, npol] c64 or c128
 * vis = sum_c flux[c] * exp(-2 pi i (u l + v m + w (n-1)))   (no 1/n)
 */
int sdp_hip_dft_point_v00(int ncomp, const double *direction_cosines,
                          const void *fluxes, int flux_nchan, int npol,
                          int64_t nrow, int nchan, const double *uvw_lambda,
                          void *vis, int vis_dtype, void *stream,
                          char *errbuf, size_t errbuf_len);

/* Same contraction with uvw in metres [nrow, 3] + freq [nchan]: the lambda
 * scaling (reference visibility/base.py:54-56) is fused into the kernel so
 * the [nrow, nchan, 3] uvw_lambda array is never materialised. */
int sdp_hip_dft_point_metres(int ncomp, const double *direction_cosines,
                             const void *fluxes, int flux_nchan, int npol,
                             int64_t nrow, int nchan, const double *uvw,
                             const double *freq, void *vis, int vis_dtype,
                             void *stream, char *errbuf, size_t errbuf_len);

/*
 * Convolution-function (AW-projection) gridder/degridder, replacing the
 * Python triple loops of grid_visibility_to_griddata /
 * degrid_visibility_from_griddata (reference
 * src/ska_sdp_func_python/grid_data/gridding.py:160-255, :502-590).
 * The Python layer evaluates the reference's WCS mappings
 * (spatial_mapping, gridding.py:60-157) into integer indices; the kernels do
 * the per-visibility slice add / einsum, including the edge-skip rule
 * (gridding.py:230-237).
 *   pu,pv,pwc,pdu,pdv [nchan_vis, nrowvis] int32 (per channel mappings)
 *   vis,wt            [nrowvis, nchan_vis, npol] c128 / f64 (flagged)
 *   cf                [cf_nchan, npol, nw, ndv, ndu, gv, gu] c128
 *   grid              [g_nchan, npol, ny, nx] c128 (accumulated)
 *   vis_to_im         [nchan_vis] int32
 *   sumwt             [g_nchan, npol] f64 (accumulated)
 *   nskipped          [1] int64 (accumulated count of edge-skipped rows)
 */
int sdp_hip_grid_cf(int64_t nrowvis, int nchan_vis, int npol,
                    const int32_t *pu, const int32_t *pv, const int32_t *pwc,
                    const int32_t *pdu, const int32_t *pdv,
                    const int32_t *vis_to_im, const void *vis,
                    const double *wt, const void *cf, int cf_nchan, int nw,
                    int ndv, int ndu, int gv, int gu, void *grid,
                    int g_nchan, int ny, int nx, double *sumwt,
                    int64_t *nskipped, void *stream, char *errbuf,
                    size_t errbuf_len);
int sdp_hip_degrid_cf(int64_t nrowvis, int nchan_vis, int npol,
                      const int32_t *pu, const int32_t *pv,
                      const int32_t *pwc, const int32_t *pdu,
                      const int32_t *pdv, const int32_t *vis_to_im,
                      const void *grid, int g_nchan, int ny, int nx,
                      const void *cf, int cf_nchan, int nw, int ndv, int ndu,
                      int gv, int gu, void *vis_out, int64_t *nskipped,
                      void *stream, char *errbuf, size_t errbuf_len);

/*
 * Batched iterative-substitution gain solver, replacing
 * _solve_with_mask + _solve_antenna_gains_itsubs_scalar / _matrix /
 * _nocrossdata + the residual functions (reference
 * src/ska_sdp_func_python/calibration/solvers.py:148-539).  One solve = one
 * gain-table row; all of its channels (and 2x2 components) iterate together
 * and stop on max|g - g_last| over antennas AND channels (solvers.py:268,
 * :427), as in the reference.
 *   baselines   canonical: a1 < a2, sorted by (a1, a2); row_start[nants+1]
 *               is the CSR offset of each a1, ant2[nbl] the partner
 *   xb, wb      [nsolve, nbl, nchan, npol] c128 / f64: the weighted sums
 *               sum(V w) and sum(w) of solvers.py:99-107 (point-source vis)
 *   gain        [nsolve, nants, nchan, nrec, nrec] c128 (in: start, out)
 *   gwt         [nsolve, nants, nchan, nrec, nrec] f64   (out)
 *   residual    [nsolve, nchan, nrec, nrec] f64          (out)
 *   niter_out   [nsolve] int32 iterations used (niter + 1: not converged)
 * mode: 0 scalar (npol 1), 1 matrix (npol 4, crosspol), 2 no cross data
 * (npol 2, or npol 4 without crosspol).
 */
int sdp_hip_solve_gains(int nsolve, int nants, int nbl, const int32_t *row_start,
                        const int32_t *ant2, int nchan, int npol, int mode,
                        const void *xb, const double *wb, void *gain, double *gwt,
                        double *residual, int32_t *niter_out, int niter, double tol,
                        int phase_only, int refant, double damping, void *stream,
                        char *errbuf, size_t errbuf_len);

/*
 * Calibration neighbours of StefCal.  Visibility
 * arrays are the Visibility's [ntimes, nbl, nchan, npol] in C order:
 * vis / model c64 or c128 (vis_dtype), weight f64, flags integers of
 * flag_bytes (1, 4, 8) or NULL; model_flags (same type) masks the model
 * where the model Visibility carries flags of its own (NULL: the vis flags).
 *
 * sdp_hip_point_sums: divide_visibility (reference
 * src/ska_sdp_func_python/visibility/operations.py:145-189; model may be
 * NULL = no division) fused with solve_gaintable's per-gain-row sums
 * (calibration/solvers.py:82-107):
 *   x_b[r, j, fg, p]  = sum_{t in row r} sum_{f} x * xwt * (1 - flag)
 *   xwt_b[r, j, fg, p] = sum ... xwt * (1 - flag)
 * over all channels f when nchan_g == 1, else f = fg.  Row r's vis time
 * indices are time_idx[row_ptr[r] .. row_ptr[r+1]) (device int32 CSR).
 * Output baseline j < nbl_out reads source baseline bl_perm[j] (NULL =
 * identity, nbl_out = nbl) and is conjugated where bl_conj[j] (NULL = never):
 * StefCal's canonical order.  xb c128 / xwt f64 [nrow_g, nbl_out, nchan_g,
 * npol], overwritten.
 */
int sdp_hip_point_sums(int64_t ntimes, int nbl, int nchan, int npol,
                       const void *vis, const void *model, int vis_dtype,
                       const double *weight, const void *flags,
                       const void *model_flags, int flag_bytes,
                       int nrow_g, const int32_t *row_ptr,
                       const int32_t *time_idx, int nchan_g, int nbl_out,
                       const int32_t *bl_perm, const uint8_t *bl_conj, void *xb,
                       double *xwt, void *stream, char *errbuf,
                       size_t errbuf_len);
/* divide_visibility alone over n samples: x_out = fv / fm where
 * xwt_out = |fm|^2 fw > 0, else 0 (f = flagged); x_out has vis_dtype. */
int sdp_hip_divide_vis(int64_t n, const void *vis, const void *model,
                       int vis_dtype, const double *weight, const void *flags,
                       const void *model_flags, int flag_bytes, void *x_out,
                       double *xwt_out, void *stream, char *errbuf,
                       size_t errbuf_len);
/*
 * sdp_hip_apply_gains: apply_gaintable (calibration/operations.py:23-256) in
 * place on vis / weight.  time_row[ntimes] (device int32) is the gain row
 * applied to each vis time, or -1; ant1/ant2 [nbl] int32 the baseline's
 * antennas; gain c128 [nrow_g, nants, nchan_g, nrec, nrec].  Gain channel c
 * acts on vis channel c only (channels >= nchan_g keep their values, as in
 * the reference).  npol 1: V * sum_lm g1 conj(g2) (1/g where |g| > 0 for
 * inverse), zero vis + weight where that is 0; npol 2 / 4: G1 V conj(G2)
 * (elementwise conj) with V diagonal / 2x2, inverse = the 2x2 inverses; a
 * baseline with a singular gain zeroes pol 0 (npol 2) or all pols (npol 4)
 * and their weights.  use_flags: a gain row whose window holds any set flag
 * works on the flagged vis / weights of that window.
 */
int sdp_hip_apply_gains(int64_t ntimes, int nbl, int nchan, int npol,
                        void *vis, int vis_dtype, double *weight,
                        const void *flags, int flag_bytes, int use_flags,
                        const int32_t *ant1, const int32_t *ant2,
                        const int32_t *time_row, const void *gain, int nrow_g,
                        int nants, int nchan_g, int nrec, int inverse,
                        void *stream, char *errbuf, size_t errbuf_len);

/*
 * Imaging weights, replacing the Python row loops of
 * grid_visibility_weight_to_griddata (reference
 * src/ska_sdp_func_python/grid_data/gridding.py:258-334) and
 * griddata_visibility_reweight (:362-499), which weight_visibility
 * (src/ska_sdp_func_python/imaging/weighting.py:35-68) chains, and the two
 * tapers (weighting.py:71-136).
 *   uvw          [nrow, 3] f64 metres (nrow = ntimes * nbaselines)
 *   freq         [nchan] f64 Hz
 *   weight       [nrow, nchan, npol] f64 (the Visibility's weight)
 *   flags        [nrow, nchan, npol] integers of flag_bytes (1, 4 or 8) or
 *                NULL; flagged weight = weight * (1 - flags) as in the
 *                datamodels' flagged_weight
 *   vis_to_im    [nchan] int32 image channel of each visibility channel
 *   grid_wcs     [6] f64: crval, cdelt, crpix of the GridData's UU axis, then
 *                of its VV axis; cell = round((uv - crval) / cdelt + crpix - 1)
 *   grid         [g_nchan, npol, ny, nx] f64: real part of the GridData
 *   npol         1, 2 or 4
 */
/* Accumulates the flagged weight into grid at the sample's cell and at its
 * conjugate's; sumwt [g_nchan, npol] += 2 * weight; rows whose cell or
 * conjugate cell is off the grid add npol to *nskipped (int64, accumulated). */
int sdp_hip_grid_weights(int64_t nrow, int nchan, int npol, const double *uvw,
                         const double *freq, const double *weight,
                         const void *flags, int flag_bytes,
                         const int32_t *vis_to_im, const double *grid_wcs,
                         double *grid, int g_nchan, int ny, int nx,
                         double *sumwt, int64_t *nskipped, void *stream,
                         char *errbuf, size_t errbuf_len);
/* weighting 0 natural (imaging_weight = weight), 1 uniform (flagged weight /
 * grid weight), 2 robust (flagged weight / (1 + f2 * grid weight), f2 =
 * robust_coef * sum(sumwt) / sum(grid^2), robust_coef = (5 * 10^-robustness)^2;
 * sumwt NULL means 2 * sum of flagged weights).  imaging_weight
 * [nrow, nchan, npol] f64 is overwritten (it is read only where the grid
 * weight is NaN, as the reference keeps the flagged imaging weight there). */
int sdp_hip_reweight(int64_t nrow, int nchan, int npol, const double *uvw,
                     const double *freq, const double *weight,
                     const void *flags, int flag_bytes,
                     const int32_t *vis_to_im, const double *grid_wcs,
                     const double *grid, int g_nchan, int ny, int nx,
                     int weighting, double robust_coef, const double *sumwt,
                     int n_sumwt, double *imaging_weight, void *stream,
                     char *errbuf, size_t errbuf_len);
/* imaging_weight = flagged imaging weight * taper(row, chan), in place.
 * kind 0 gaussian: exp(-param * |uv|^2 / lambda^2), param = pi^2 beam^2 / (4 ln 2);
 * kind 1 tukey: tukey_filter(|uv| / max|uv|, param). */
int sdp_hip_taper(int64_t nrow, int nchan, int npol, const double *uvw,
                  const double *freq, const void *flags, int flag_bytes,
                  int kind, double param, double *imaging_weight, void *stream,
                  char *errbuf, size_t errbuf_len);

#ifdef __cplusplus
}
#endif
#endif /* SKA_SDP_HIP_H */
