/*
 * m3s_match.h — C ABI of the MI355X matching kernels of MASt3R-SLAM.
 *
 * Drop-in for the two non-GN entry points of the reference's
 * `mast3r_slam_backends` module (gn.cpp:84-114, declared gn.h:89-116; kernels
 * matching_kernels.cu), called by matching.py:60-85:
 *
 *   iter_proj       per-pixel Levenberg-Marquardt projection of a 3D ray onto
 *                   a ray image with gradients (matching_kernels.cu:119-296)
 *   refine_matches  dilated local search maximising the descriptor dot
 *                   product (matching_kernels.cu:25-116)
 *
 * Plain C: device pointers, sizes, the caller's hipStream_t as `void *`, an
 * int status (M3S_OK / M3S_EINVAL / M3S_ELAUNCH of m3s_gn.h). All tensors are
 * the reference's layouts, contiguous, on the device. One launch each, no host
 * synchronisation, no allocation.
 */
#ifndef M3S_MATCH_H
#define M3S_MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct m3s_iter_proj_args {
  const float *rays_img;    /* [B, H, W, 9]: unit ray (3), d/du (3), d/dv (3) */
  const float *pts_3d_norm; /* [B, N, 3]: unit rays to project               */
  const float *p_init;      /* [B, N, 2]: initial pixel (u, v)               */
  int64_t B, H, W, N;
  int max_iter;
  float lambda_init;
  float cost_thresh;
  float *p_new;       /* [B, N, 2] out                                       */
  uint8_t *converged; /* [B, N] out (torch.bool)                             */
} m3s_iter_proj_args;

/* Replaces iter_proj (gn.cpp:84-99 -> matching_kernels.cu:119-296). */
int m3s_iter_proj(const m3s_iter_proj_args *a, void *stream);

#define M3S_DESC_F16 0 /* D11/D21 are float16 (the reference's .half() call) */
#define M3S_DESC_F32 1

typedef struct m3s_refine_args {
  const void *D11;   /* [B, H, W, F] descriptors of image 1             */
  const void *D21;   /* [B, N, F] descriptors of the pixels to refine   */
  const int64_t *p1; /* [B, N, 2] current match (u, v) in image 1       */
  int64_t B, H, W, N, F;
  int dtype;        /* M3S_DESC_F16 or M3S_DESC_F32                      */
  int radius;       /* matching.radius (3)                               */
  int dilation_max; /* matching.dilation_max (5)                         */
  int64_t *p1_new;  /* [B, N, 2] out                                     */
} m3s_refine_args;

/* Replaces refine_matches (gn.cpp:101-114 -> matching_kernels.cu:25-116). */
int m3s_refine_matches(const m3s_refine_args *a, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* M3S_MATCH_H */
