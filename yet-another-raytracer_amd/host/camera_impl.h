/* camera_impl.h — Camera::new (camera.rs:39-80), host arithmetic shared by libyart and
 * libyart_host. f64, no FMA contraction (both libraries build with -ffp-contract=off). */
#ifndef YART_CAMERA_IMPL_H
#define YART_CAMERA_IMPL_H

#include <math.h>
#include "../../include/yart.h"

static inline void yart_cam_sub(const double a[3], const double b[3], double o[3]) {
  o[0] = a[0] - b[0]; o[1] = a[1] - b[1]; o[2] = a[2] - b[2];
}
static inline double yart_cam_len(const double a[3]) { return sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]); }
static inline void yart_cam_unit(const double a[3], double o[3]) { /* vec3.rs:203-211 */
  o[0] = a[0] / yart_cam_len(a); o[1] = a[1] / yart_cam_len(a); o[2] = a[2] / yart_cam_len(a);
}
static inline void yart_cam_cross(const double a[3], const double b[3], double o[3]) { /* vec3.rs:225-233 */
  o[0] = a[1] * b[2] - a[2] * b[1]; o[1] = a[2] * b[0] - a[0] * b[2]; o[2] = a[0] * b[1] - a[1] * b[0];
}

static inline int yart_camera_init_impl(yart_camera* c, const double lookfrom[3], const double lookat[3],
                                        const double vup[3], double vfov, double aspect, double aperture,
                                        double focus_dist, double time0, double time1) {
  if (!c || !lookfrom || !lookat || !vup) return YART_ERR_INVALID;
  const double PI = 3.141592653589793;
  double theta = vfov * PI / 180.0;            /* degrees_to_radians camera.rs:35-37 */
  double h = tan(theta / 2.0);
  double viewport_height = 2.0 * h;
  double viewport_width = aspect * viewport_height;
  double d[3], w[3], uu[3], u[3], v[3];
  yart_cam_sub(lookfrom, lookat, d);
  yart_cam_unit(d, w);
  yart_cam_cross(vup, w, uu);
  yart_cam_unit(uu, u);
  yart_cam_cross(w, u, v);
  for (int i = 0; i < 3; ++i) {
    c->origin[i] = lookfrom[i];
    c->horizontal[i] = focus_dist * viewport_width * u[i];   /* (fd * vw) * u */
    c->vertical[i] = focus_dist * viewport_height * v[i];
    c->u[i] = u[i]; c->v[i] = v[i]; c->w[i] = w[i];
  }
  /* origin - horizontal / 2.0 - vertical / 2.0 - focus_dist * w (Div<f64> by a non-zero 2.0) */
  for (int i = 0; i < 3; ++i)
    c->lower_left_corner[i] = c->origin[i] - c->horizontal[i] / 2.0 - c->vertical[i] / 2.0 - focus_dist * w[i];
  c->lens_radius = aperture / 2.0;
  c->time0 = time0;
  c->time1 = time1;
  return YART_OK;
}

#endif
