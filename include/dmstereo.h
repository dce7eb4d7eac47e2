/*
 * dmstereo.h -- C ABI of the MI355X (gfx950) DeepMatching stereo correlation engine.
 *
 * The reference path this ABI replaces is Python (Yuki-Kumon/deepmatching_stereo_matching):
 *   misc/Correlation_map.py  Correlation_map (:29-173), Maxpool (:176-184)
 *   misc/Feature_value.py    Feature_value (:18-43) -> cv2.matchTemplate + min_max
 *   misc/Matching.py         Matching (:20-255), Zero_padding (:258-268)
 *   misc/Calc_difference.py  Calc_difference.cal_map (:26-49)
 *   misc/sub_pix_cal.py      sub_pix_cal (:22-53)
 *   misc/image_cut_solver.py ImageCutSolver._execute_matching stitching (:144-179)
 *   misc/optimize_loop.py    optimize_loop (:15-37), image_threshold (:40-44)
 *   misc/opt_loop.py         optimize_loop_bilateral_* (:16-58), make_weight (:60-85)
 * The Python mirror of that surface (deepmatching_stereo_matching_amd/misc/) binds
 * these entry points with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every pointer argument named d_* is DEVICE memory owned by the caller (torch
 *    tensors in the Python host).  The library never allocates or frees device memory
 *    and keeps no global mutable state besides a per-thread error string.
 *  - Work is enqueued on `stream` (a hipStream_t passed as void*; NULL = default stream)
 *    and is asynchronous; nothing here synchronises.
 *  - Return 0 (DM_OK) or a negative dm_status; dm_last_error() describes the failure.
 *
 * Shapes.  A batch holds T tiles of equal size cut from one image pair.  For tile t the
 * crop is rows [org_t.r, org_t.r + h0 + ws - 1) x cols [org_t.c, org_t.c + w0 + ws - 1) of
 * img1 and img2 (the same window in both, as ImageCutSolver._cut_and_pool does,
 * image_cut_solver.py:95-113).  h0 = H' and w0 = W' are the correlation-map sides
 * (Correlation_map: H' = H - 2*exclusive_pix).  P = h0*w0.
 *  level 0  : "co_map", float32 [T][P][P] (min-max normalised, NOT rectified)
 *  level l>0: float64 [T][Pl][Pl], Pl = (h0>>l)*(w0>>l), rectified (**1.4) like
 *             co_map_list[l].
 */
#ifndef DMSTEREO_H
#define DMSTEREO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum dm_status {
    DM_OK = 0,
    DM_ERR_ARG = -1,         /* bad pointer / size argument                              */
    DM_ERR_SHAPE = -2,       /* shape the reference cannot process (even ws, odd sides) */
    DM_ERR_UNSUPPORTED = -3, /* valid for the reference, not (yet) for this engine      */
    DM_ERR_HIP = -4          /* a HIP runtime call failed                               */
};

enum dm_method { /* cv2 constants, Feature_value.py:23-30 */
    DM_TM_CCOEFF = 4,
    DM_TM_CCOEFF_NORMED = 5
};

enum dm_cal_mode { /* Calc_difference.cal_map modes, Calc_difference.py:30 */
    DM_CAL_ELEVATION = 0,  /* j - map[1] */
    DM_CAL_ELEVATION2 = 1, /* i - map[0] */
    DM_CAL_DISTANCE = 2    /* || (i, j) - map[:2] || */
};

typedef struct dm_tiles {
    const uint8_t *d_img1;    /* "img" / original / before   (Correlation_map arg 1) */
    const uint8_t *d_img2;    /* "template" / after          (Correlation_map arg 2) */
    int32_t pitch1, pitch2;   /* row pitch in bytes                                   */
    const int32_t *d_origins; /* [T][2] crop top-left (row, col)                      */
    int32_t T;                /* tiles in the batch                                    */
    int32_t h0, w0;           /* correlation-map sides                                 */
    int32_t ws;               /* window_size, odd, 1..15                               */
    int32_t method;           /* dm_method                                             */
} dm_tiles;

/* Size in bytes of the per-batch statistics workspace: per-patch / per-window moments and
 * the per-patch min/max of the level-0 map (6 * 4 * T * P), plus, for shapes the MFMA
 * kernels take, the window operands in MFMA fragment order (T * h0 * (w0/16) * (KS*1024
 * + 128), KS = ceil(ws^2 / 64)), and for ws <= 5 a second such region in the volume
 * kernels' column-group layout (dm_corr_volume and dm_corr_volume_f16 fill it themselves). */
size_t dm_stats_bytes(const dm_tiles *b);

/* Per-patch and per-window moments.
 * Replaces Correlation_map._create_atomic_patch (Correlation_map.py:51-67) and the
 * template/window sums inside cv2.matchTemplate (Feature_value.py:41). */
int dm_corr_stats(const dm_tiles *b, void *d_stats, void *stream);

/* Level-0 ZNCC + per-patch min-max + rectification + MaxPool(3,2,1) + 4-child average +
 * rectification, fused: writes level 1 (float64 [T][P1][P1]) and the per-patch min/max
 * into d_stats.  Level 0 is never written.
 * Replaces Correlation_map._create_simple_initial_co_map (:69-87), Feature_value.min_max
 * (Feature_value.py:32-37), _rectification (:158-159) and the first _aggregation
 * (:89-130) of _multi_level_correlation_pyramid (:132-156).  Needs dm_corr_stats first. */
int dm_corr_level1(const dm_tiles *b, void *d_stats, double *d_level1, void *stream);

/* dm_corr_level1 followed by the second _aggregation (Correlation_map.py:89-130, :148-153)
 * in the same kernel: writes level 2 (float64 [T][P2][P2], P2 = (h0/4)*(w0/4)) and, when
 * d_level1 is non-NULL, level 1 as well.  With d_level1 NULL level 1 never reaches HBM;
 * dm_match then evaluates it on demand.  Needs h0 % 4 == 0, w0 in {32,64,128,256},
 * ws <= 15 (DM_ERR_UNSUPPORTED otherwise: use dm_corr_level1 + dm_aggregate). */
int dm_corr_level12(const dm_tiles *b, void *d_stats, double *d_level1, double *d_level2, void *stream);

/* Materialise the level-0 min-max volume "co_map" (float32 [T][P][P]) and the per-patch
 * min/max.  Replaces _create_simple_initial_co_map (:69-87) for callers that read
 * co_map directly (bad_matching.py:62-70).  Needs dm_corr_stats first. */
int dm_corr_volume(const dm_tiles *b, void *d_stats, float *d_l0, void *stream);

/* dm_corr_volume with a binary16 volume (uint16_t bit patterns, [T][P][P]): each float32
 * co_map value rounded to nearest-even half, i.e. np.float16(co_map).  The fp16
 * correlation volume of BASELINE config C5 (2 B/voxel instead of 4); not bit-exact with
 * the reference by construction (SURVEY.md 8(a) parity rules: a flip rate is reported).
 * Needs dm_corr_stats first. */
int dm_corr_volume_f16(const dm_tiles *b, void *d_stats, uint16_t *d_l0, void *stream);

/* Flags of dm_corr_volume_ex. */
enum {
    DM_VOLUME_F16 = 1,            /* binary16 output (dm_corr_volume_f16), else float32     */
    DM_VOLUME_MINMAX_KNOWN = 2    /* d_stats already holds the per-patch min/max: written by
                                     dm_corr_level1 / dm_corr_level12 / a volume call on the
                                     same tiles and stats.  The kernel then skips its own
                                     min/max sweep (the same values: bit-identical output).  */
};

/* dm_corr_volume / dm_corr_volume_f16 with flags: the same level-0 volume, and, with
 * DM_VOLUME_MINMAX_KNOWN, without re-deriving the per-patch min/max that an earlier call
 * left in d_stats -- the reference's co_map read after Correlation_map()() has built the
 * pyramid (bad_matching.py:62-70 reads it before; Correlation_map.py:69-87 computes both
 * in one pass).  d_l0: float * or uint16_t * by DM_VOLUME_F16. */
int dm_corr_volume_ex(const dm_tiles *b, void *d_stats, int32_t flags, void *d_l0, void *stream);

/* d_out[i] = (double)half(d_in[i]) ** 1.4: _rectification (:158-159) of an fp16 volume. */
int dm_rectify_f16(const uint16_t *d_in, size_t n, double *d_out, void *stream);

/* d_out[i] = d_in[i] ** 1.4 (pinned float64 pow, dm_pow.h).  Replaces
 * Correlation_map._rectification (:158-159) for the materialised co_map_list[0]. */
int dm_rectify(const float *d_in, size_t n, double *d_out, void *stream);

/* Same for float64 input (Correlation_map._rectification on an aggregated map). */
int dm_rectify64(const double *d_in, size_t n, double *d_out, void *stream);

/* Self-test of the pow14 forms the fused kernels evaluate in place of _rectification
 * (:158-159), tables in LDS as the kernels hold them.  d_out[i] = form(d_in[i]); each form
 * equals dm_pow14 (dm_pow.h) bit for bit on its domain, and only there:
 *   DM_POW_F32   pow14_zf((float)x): 0, NaN and float32-normal x in (0, 1] (the level
 *                kernel's child values: x is a float32 in [0, 1] or NaN)
 *   DM_POW_Q4    pow14_q4(s) = pow14(s / 4): s == 0, NaN, or s / 4 in [2^-319, 1] (a sum of
 *                four children, level-1 / level-2 averaging); 0 < s / 4 < 2^-319 gives 0 and
 *                s = +inf NaN instead of dm_pow14's values
 *   DM_POW_K     pow14_k(x): 0, NaN and x in [2^-319, 1]
 *   DM_POW_FULL  pow14_lds(x): every double (the slow path outside [2^-319, 1])
 *   DM_POW_Q4G   pow14_q4g(s), DM_POW_KG pow14_kg(x) (ABI 1.10): the same as DM_POW_Q4 / DM_POW_K
 *                bit for bit on EVERY double, from the float32-exponent table rows instead of
 *                the float64 ones (the pruned level kernel, whose LDS holds no gz rows) */
enum dm_pow_variant { DM_POW_F32 = 0, DM_POW_Q4 = 1, DM_POW_K = 2, DM_POW_FULL = 3, DM_POW_Q4G = 4, DM_POW_KG = 5 };
int dm_pow14_variant(int32_t variant, const double *d_in, size_t n, double *d_out, void *stream);

/* One pyramid step for levels >= 1: MaxPool2d(3,2,1) per map, (ul+ur+ll+lr)/4, and
 * (rectify != 0) the 1.4 power.  d_in float64 [T][h*w][h*w] -> d_out float64
 * [T][(h/2)*(w/2)][(h/2)*(w/2)].
 * Replaces Correlation_map._aggregation (:89-130) [+ _rectification (:148)]. */
int dm_aggregate(const double *d_in, int32_t T, int32_t h, int32_t w, int32_t rectify,
                 double *d_out, void *stream);

/* Coarse-to-fine matching on a pyramid of nlev levels of T tiles with level-0 sides
 * h0 x w0.  d_levels is a HOST array of nlev device pointers to float64 rectified levels
 * (co_map_list).  d_levels[0] may be NULL: level 0 is then evaluated on demand from the
 * images and the statistics (b and d_stats required; b->T/h0/w0 must match).  When
 * d_levels[0] is NULL and nlev >= 3, d_levels[1] may be NULL as well (level 1 on demand,
 * for a pyramid built by dm_corr_level12 without level 1).
 * filter_num > 0 runs Matching._filter (:224-255; filter_mode 0 average, 1 median, window
 * filter_window <= 7, square maps only) after the top level and after each _B step while
 * the count lasts, as Matching._initial_move_map / _B do.
 * d_scratch: float64 [T][3][h0*w0].  d_out: float64 [T][3][h0][w0] = (row, col, score),
 * as returned by Matching.__call__ (Matching.py:211-222): _initial_move_map (:80-96),
 * _B/_calc_match (:98-149), _calc_near_match (:58-78), _sub_pix_cal (:177-209). */
int dm_match(const dm_tiles *b, const void *d_stats, const double *const *d_levels,
             int32_t nlev, int32_t T, int32_t h0, int32_t w0, int32_t sub_pix,
             int32_t filter_window, int32_t filter_num, int32_t filter_mode,
             double *d_scratch, double *d_out, void *stream);

/* Matching._sub_pix_cal (Matching.py:177-209) for a descent that stops ABOVE level 0 (an
 * N_map whose halvings end before the list does, Matching.py:85-96, :133-134): the final
 * map of a coarser level (float64 [T][3][hm][wm], from dm_match on co_map_list[bottom:]
 * without sub_pix) is refined in place against the materialised level 0 d_level0 (float64
 * [T][h0*w0][h0*w0], co_map_list[0]) at patch (i, j) and window (row, col) of each entry, as
 * the reference does; bounds are level 0's (h0, w0).  Any map is accepted and indexed as numpy
 * indexes co_map_list[0] (Matching.py:186-188, :199-201): c = int(entry), an index in [-N, N)
 * is valid and a negative one wraps, any other raises IndexError and takes the bare except
 * (:193-194, :205-206: i - d_x, j - d_y).  hm <= h0, wm <= w0.  dm_match's own sub_pix is
 * this with hm = h0, wm = w0. */
int dm_subpix_map(const double *d_level0, int32_t T, int32_t h0, int32_t w0, int32_t hm, int32_t wm,
                  double *d_map, void *stream);

/* The same refinement with level 0 evaluated on demand (ABI 1.9): the five level-0 values an
 * entry reads are recomputed from the tile batch's images and the statistics workspace of
 * dm_corr_stats + dm_corr_level1/12 (its per-patch min / max), exactly as dm_match's own
 * sub-pixel step does, so a descent that stops above level 0 never materialises
 * co_map_list[0] (T * (h0 w0)^2 float64).  d_map: float64 [b->T][3][hm][wm], in place. */
int dm_subpix_map_tiles(const dm_tiles *b, const void *d_stats, int32_t hm, int32_t wm, double *d_map,
                        void *stream);

/* misc/sub_pix_cal.py sub_pix_cal (:22-53): clamp to [-3,3], quadratic refinement of an
 * (h, w) disparity map along `direction` (0 rows, 1 cols) on the score map scaled by
 * `ratio`, reject |delta| > 1, clamp again.  float64 in/out, device pointers. */
int dm_sub_pix_cal(const double *d_arr, const double *d_score, int32_t h, int32_t w,
                   int32_t direction, double ratio, double *d_out, void *stream);

/* Calc_difference.cal_map (Calc_difference.py:26-49) on T maps [T][3][h][w] -> [T][h][w]. */
int dm_cal_map(const double *d_map, int32_t T, int32_t h, int32_t w, int32_t mode,
               double *d_out, void *stream);

/* ImageCutSolver stitching (image_cut_solver.py:144-179): tiles t = j*n0 + i of d_match
 * ([T][3][h0][w0]) are written at (stride0*i, stride1*j), later tiles overwriting
 * earlier ones.  d_dmap: [nmodes][Hout][Wout] (cal_map of each mode in `modes`, a HOST
 * array), d_score: [Hout][Wout] (map[2]).  Hout = stride0*(n0-1)+h0, likewise Wout.
 * Output cells no tile covers are NaN (np.empty garbage in the reference). */
int dm_stitch(const double *d_match, int32_t n0, int32_t n1, int32_t h0, int32_t w0,
              int32_t stride0, int32_t stride1, const int32_t *modes, int32_t nmodes,
              double *d_dmap, double *d_score, void *stream);

/* ---- Gauss-Seidel post-processing (dm_postproc.hip) -------------
 * misc/optimize_loop.py (optimize_loop :15-37, image_threshold :40-44) and misc/opt_loop.py
 * (optimize_loop_bilateral_horizon :16-35, _vertical :39-58, make_weight :60-85).  Maps are
 * float64 row-major h x w; `size` = (s0, s1) <= (h, w) bounds the sweeps as in the
 * reference; excl = `exclusion` (e).  A sweep updates the (s0-2e-1) x (s1-2e-1) cells of
 * its fixed reference order in place; here it runs as dependency levels (dm_gs_schedule)
 * and gives the sequential loops' float64 results bit for bit. */
enum dm_gs_kind {
    DM_GS_FWD4 = 0,  /* optimize_loop forward sweep, 4-neighbour (optimize_loop.py:18-25)          */
    DM_GS_BWD4 = 1,  /* optimize_loop backward sweep, with the reference's row alternation (:27-36) */
    DM_GS_BILAT = 2  /* optimize_loop_bilateral_*, (2e+1)^2 window (opt_loop.py:23-35)              */
};

/* HOST function (no device work): the dependency-level schedule of one sweep.  n =
 * max(0, s0-2e-1) * max(0, s1-2e-1) updates; order[n] receives the update sequence indices
 * grouped by level, level_off[n_levels + 1] (capacity n + 1) the level boundaries.  An
 * update's level exceeds those of the last writers of every cell it reads and of every
 * reader of its own cell since that cell's last write, so one level's updates are
 * independent and the sequential order's values are reproduced exactly. */
int dm_gs_schedule(int32_t kind, int32_t h, int32_t w, int32_t s0, int32_t s1, int32_t excl,
                   int32_t *order, int32_t *level_off, int32_t *n_levels);

/* image_threshold (optimize_loop.py:40-44): out = min(max(in, lo), hi) as two np.where
 * (NaN passes through).  In place allowed. */
int dm_image_threshold(const double *d_in, size_t n, double lo, double hi, double *d_out,
                       void *stream);

/* optimize_loop (optimize_loop.py:15-37) on an already thresholded map d_img (in place):
 * forward sweep then backward sweep of d = (-a x + alpha (L+R+U+D)) / (-a + 4 alpha),
 * a = coefficient[i, j] (d_coef hc x wc).  Schedules from dm_gs_schedule (DM_GS_FWD4,
 * DM_GS_BWD4) in device memory.  d_diff: n float64 scratch; *d_error = the backward
 * sweep's sum of |x - d| in sequence order. */
int dm_optimize_loop(double *d_img, const double *d_coef, int32_t hc, int32_t wc, int32_t h,
                     int32_t w, int32_t s0, int32_t s1, int32_t excl, double alpha,
                     const int32_t *d_fwd_order, const int32_t *d_fwd_off, int32_t fwd_levels,
                     const int32_t *d_bwd_order, const int32_t *d_bwd_off, int32_t bwd_levels,
                     double *d_diff, double *d_error, void *stream);

/* make_weight (opt_loop.py:60-85): d_gauss[(2e+1)^2] = exp(-(dy^2+dx^2) / den_space),
 * d_color[s0-e][s1-e][2e+1][2e+1] = exp(-(c^2) / den_color) with c = guide[i,j] -
 * guide[i+dy, j+dx] on the filled cells, 0 elsewhere.  den_* = 2.0 * sigma[k]**2 as the
 * caller's Python evaluates it.  exp is the pinned dm_exp (csrc/dm_exp.h). */
int dm_make_weight(const double *d_guide, int32_t h, int32_t w, int32_t s0, int32_t s1,
                   int32_t excl, double den_color, double den_space, double *d_gauss,
                   double *d_color, void *stream);

/* optimize_loop_bilateral_horizon (vertical = 0) / _vertical (1) (opt_loop.py:16-58):
 * one sweep of d = (-a b + sum(g cw sub)) / (-a + sum(g cw)) in place on d_img, weights
 * from dm_make_weight, coefficients coefficient[e, e] and [e, e+-1] / [e+-1, e] of d_coef
 * (hc x wc), numpy's pairwise sum order.  Schedule: dm_gs_schedule(DM_GS_BILAT).
 * *d_error = sum of |x - d| in sequence order; d_diff: n float64 scratch. */
int dm_opt_loop_bilateral(double *d_img, const double *d_color, const double *d_gauss,
                          const double *d_coef, int32_t hc, int32_t wc, int32_t h, int32_t w,
                          int32_t s0, int32_t s1, int32_t excl, int32_t vertical,
                          const int32_t *d_order, const int32_t *d_off, int32_t n_levels,
                          double *d_diff, double *d_error, void *stream);

/* Sum of d_v[0..n) in sequence order, the float64 loop `error += v` of
 * misc/optimize_loop.py:34 / misc/opt_loop.py:33 bit for bit, for terms >= 0 (NaN and inf
 * propagate as in the loop).  Computed as exact integer prefix sums between the steps where
 * the running sum climbs a binade or a tie occurs (dm_postproc.hip, k_seq_sum_seg).  *d_out
 * (device) receives the sum; n == 0 gives +0.  The post-processing entries use it for their
 * error sums. */
int dm_seq_sum(const double *d_v, int64_t n, double *d_out, void *stream);

/* The compile-time kernel switches this library was built with ("S1=1 C2_NB=4 ..."; see
 * dm_kernels.hip: DM_S1, DM_C*_NB, DM_VL_*), which decide the kernel instance each shape
 * launches -- tools/kernel_hash.py derives the profiled instances' symbols from it. */
const char *dm_build_config(void);

/* Human-readable description of the last failure on this thread. */
const char *dm_last_error(void);

/* ABI version (major * 100 + minor): 110 (1.1 adds dm_corr_level12, 1.2 the fp16 volume
 * dm_corr_volume_f16 / dm_rectify_f16, 1.3 the Gauss-Seidel post-processing, 1.4 a larger
 * stats workspace: a second window-operand region for the volume kernels, window stats
 * carried inside the operand tiles, 1.5 dm_corr_volume_ex, 1.6 dm_pow14_variant and the
 * 4-tile column groups of dm_corr_stats' window operands at S = 128 / 256, 1.7 dm_seq_sum,
 * 1.8 dm_subpix_map, 1.9 dm_subpix_map_tiles and the row-pair strips of dm_corr_stats'
 * workspace for the level kernel's min / max sweep, 1.10 the DM_POW_Q4G / DM_POW_KG forms of
 * dm_pow14_variant). */
int dm_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* DMSTEREO_H */
