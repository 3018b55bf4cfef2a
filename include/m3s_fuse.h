/*
 * m3s_fuse.h — C ABI of the MI355X kernels on either side of the GN/matching
 * path (SURVEY.md §8f "next" #2 and #4):
 *
 *   m3s_fuse_pointmap  keyframe pointmap fusion after tracking:
 *                      X_kf <- filter(X_kf, C_kf, T_CkCf . X_f, C_f)
 *                      (tracker.py:98-99 + Frame.update_pointmap, frame.py:41-100),
 *                      the Sim(3) act fused into the filter, one pass over HBM.
 *   m3s_prep_rays      the inputs of iter_proj from two pointmaps
 *                      (prep_for_iter_proj, matching.py:25-49, with the Scharr
 *                      ray-image gradient of image.py:5-38), one pass.
 *
 * Plain C: device pointers, sizes, the caller's hipStream_t as `void *`, an int
 * status (M3S_OK / M3S_EINVAL / M3S_ELAUNCH of m3s_gn.h). One launch each, no
 * host synchronisation, no allocation.
 */
#ifndef M3S_FUSE_H
#define M3S_FUSE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define M3S_FILTER_WEIGHTED_POINTMAP 0 /* frame.py:73-76 (config default) */
#define M3S_FILTER_INDEP_CONF 1        /* frame.py:68-72                  */
#define M3S_FILTER_RECENT 2            /* frame.py:59-62: overwrite       */
#define M3S_FILTER_WEIGHTED_SPHERICAL 3 /* frame.py:78-100: confidence-weighted
                                           mean of (r, phi, theta)          */

typedef struct m3s_fuse_args {
  float *X_canon;      /* [HW, 3] keyframe canonical pointmap, updated in place */
  float *C;            /* [HW] keyframe accumulated confidence, in place        */
  const float *X_new;  /* [HW, 3] new points (frame points matched to KF pixels)*/
  const float *C_new;  /* [HW] their confidence                                 */
  const float *T;      /* [8] device Sim(3) applied to X_new first (T_CkCf), or NULL */
  int64_t HW;
  int mode;            /* M3S_FILTER_*                                          */
} m3s_fuse_args;

int m3s_fuse_pointmap(const m3s_fuse_args *a, void *stream);

typedef struct m3s_prep_rays_args {
  const float *X11; /* [B, H, W, 3] pointmap of view 1                         */
  const float *X21; /* [B, H*W, 3] points of view 2 in view 1's frame          */
  int64_t B, H, W;
  float *rays_img;  /* [B, H, W, 9] out: unit ray, d/du, d/dv (Scharr / 32)     */
  float *pts_norm;  /* [B, H*W, 3] out: unit rays of X21                         */
} m3s_prep_rays_args;

int m3s_prep_rays(const m3s_prep_rays_args *a, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* M3S_FUSE_H */
