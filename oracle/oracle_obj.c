/*
 * oracle_obj.c — TEST INFRASTRUCTURE ONLY: an OBJ reader of the oracle's own, independent of the
 * product's host loader (yet-another-raytracer_amd/host/scene.cpp), so the triangle arrays the
 * product renders can be checked against a second reading of the same file.
 *
 * What it restates: TriangleMesh::from_obj (raytracer/src/triangle.rs:111-174) over
 * tobj 4.0.2 (Cargo.lock) loaded with tobj::GPU_LOAD_OPTIONS (triangulate + single_index), as tobj
 * documents them:
 *   - `v x y z [w]`, `vt u [v [w]]`, `vn x y z` are parsed as f32 (tobj's default float type;
 *     Rust's f32::from_str is correctly rounded, as glibc strtof is);
 *   - `f` vertices are `v`, `v/vt`, `v//vn` or `v/vt/vn`, 1-based, negative = relative to the
 *     elements read so far;
 *   - a polygon of n vertices becomes the fan (v0, vk, vk+1), k = 1 .. n-2 (triangulate);
 *   - faces come out in file order (one model per `o`/`g` in tobj; from_obj appends the models'
 *     triangles in order, so the concatenation is the file's face order).
 * and then triangle.rs:143-163: a vertex without `vn` takes the face normal
 * (v1 - v0).cross(v2 - v0).unit_vector() (vec3.rs:204-234: unit_vector divides each component by
 * length(), so a degenerate face gives NaN), a vertex without `vt` takes (0, 0); everything is
 * widened to f64. A file whose faces mix vertices with and without `vn` (or `vt`) is refused: with
 * single_index tobj then emits per-vertex arrays that no longer line up with the indices, and the
 * reference's behaviour on such a file is an accident of that misalignment.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float* v; size_t n, cap; } fvec;

static int fpush(fvec* a, float x) {
  if (a->n == a->cap) {
    size_t c = a->cap ? 2 * a->cap : 1024;
    float* p = (float*)realloc(a->v, c * sizeof(float));
    if (!p) return -1;
    a->v = p;
    a->cap = c;
  }
  a->v[a->n++] = x;
  return 0;
}

/* one face vertex: indices into v / vt / vn (0-based), -1 = absent */
typedef struct { long v, vt, vn; } fvert;

static long resolve(long idx, size_t count) {  /* 1-based or negative-relative -> 0-based, -2 = bad */
  if (idx > 0) return (size_t)idx <= count ? idx - 1 : -2;
  if (idx < 0) return (long)count + idx >= 0 ? (long)count + idx : -2;
  return -2;
}

static int parse_fvert(const char* tok, size_t nv, size_t nvt, size_t nvn, fvert* out) {
  char* end;
  out->vt = out->vn = -1;
  long a = strtol(tok, &end, 10);
  if (end == tok) return -1;
  out->v = resolve(a, nv);
  if (out->v < 0) return -1;
  if (*end != '/') return *end == '\0' ? 0 : -1;
  const char* p = end + 1;
  if (*p != '/') {
    long b = strtol(p, &end, 10);
    if (end == p) return -1;
    out->vt = resolve(b, nvt);
    if (out->vt < 0) return -1;
    p = end;
    if (*p == '\0') return 0;
    if (*p != '/') return -1;
  }
  p++;
  long c = strtol(p, &end, 10);
  if (end == p || *end != '\0') return -1;
  out->vn = resolve(c, nvn);
  return out->vn < 0 ? -1 : 0;
}

/* Reads the file; with pos == NULL only counts. Returns 0 or a negative error. */
static int obj_read(const char* path, float* pos, double* nrm, double* uv, uint32_t cap, uint32_t* n_out) {
  FILE* f = fopen(path, "r");
  if (!f) return -5;
  fvec V = {0}, VT = {0}, VN = {0};
  char line[65536];
  uint32_t n = 0;
  int rc = 0, with_vn = -1, with_vt = -1;
  fvert* fv = NULL;
  size_t fv_cap = 0;
  while (rc == 0 && fgets(line, sizeof line, f)) {
    char* hash = strchr(line, '#');
    if (hash) *hash = '\0';
    char* save = NULL;
    char* key = strtok_r(line, " \t\r\n", &save);
    if (!key) continue;
    if (!strcmp(key, "v") || !strcmp(key, "vn") || !strcmp(key, "vt")) {
      fvec* dst = key[1] == '\0' ? &V : key[1] == 'n' ? &VN : &VT;
      const int want = key[1] == 't' ? 2 : 3;  /* vt: u, v (a missing v reads 0); w ignored */
      for (int k = 0; k < want; ++k) {
        char* t = strtok_r(NULL, " \t\r\n", &save);
        float x = 0.0f;
        if (t) {
          char* e;
          x = strtof(t, &e);
          if (e == t) { rc = -1; break; }
        } else if (!(key[1] == 't' && k == 1)) {
          rc = -1;
          break;
        }
        if (fpush(dst, x)) { rc = -3; break; }
      }
    } else if (!strcmp(key, "f")) {
      size_t m = 0;
      for (char* t; (t = strtok_r(NULL, " \t\r\n", &save));) {
        if (m == fv_cap) {
          fv_cap = fv_cap ? 2 * fv_cap : 64;
          fvert* p = (fvert*)realloc(fv, fv_cap * sizeof(fvert));
          if (!p) { rc = -3; break; }
          fv = p;
        }
        if (parse_fvert(t, V.n / 3, VT.n / 2, VN.n / 3, &fv[m])) { rc = -1; break; }
        m++;
      }
      if (rc) break;
      for (size_t i = 0; i < m; ++i) {
        const int hn = fv[i].vn >= 0, ht = fv[i].vt >= 0;
        if (with_vn < 0) with_vn = hn;
        if (with_vt < 0) with_vt = ht;
        if (with_vn != hn || with_vt != ht) { rc = -4; break; }
      }
      if (rc) break;
      for (size_t k = 1; m >= 3 && k + 1 < m; ++k) {  /* fan: (0, k, k+1) */
        if (pos) {
          if (n >= cap) { rc = -1; break; }
          const fvert* tri[3] = {&fv[0], &fv[k], &fv[k + 1]};
          double p[3][3];
          for (int c = 0; c < 3; ++c)
            for (int a = 0; a < 3; ++a) {
              const float x = V.v[3 * tri[c]->v + a];
              pos[9 * (size_t)n + 3 * c + a] = x;
              p[c][a] = (double)x;
            }
          /* default_normal = (v1 - v0).cross(v2 - v0).unit_vector() (triangle.rs:147-149) */
          const double e1[3] = {p[1][0] - p[0][0], p[1][1] - p[0][1], p[1][2] - p[0][2]};
          const double e2[3] = {p[2][0] - p[0][0], p[2][1] - p[0][1], p[2][2] - p[0][2]};
          const double cr[3] = {e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2],
                                e1[0] * e2[1] - e1[1] * e2[0]};
          const double len = sqrt(cr[0] * cr[0] + cr[1] * cr[1] + cr[2] * cr[2]);
          for (int c = 0; c < 3; ++c) {
            for (int a = 0; a < 3; ++a)
              nrm[9 * (size_t)n + 3 * c + a] = tri[c]->vn >= 0 ? (double)VN.v[3 * tri[c]->vn + a] : cr[a] / len;
            if (uv) {
              uv[6 * (size_t)n + 2 * c] = tri[c]->vt >= 0 ? (double)VT.v[2 * tri[c]->vt] : 0.0;
              uv[6 * (size_t)n + 2 * c + 1] = tri[c]->vt >= 0 ? (double)VT.v[2 * tri[c]->vt + 1] : 0.0;
            }
          }
        }
        n++;
      }
    }
    /* o, g, s, usemtl, mtllib, l, p: no triangles */
  }
  fclose(f);
  free(V.v); free(VT.v); free(VN.v); free(fv);
  if (rc) return rc;
  *n_out = n;
  return 0;
}

int oracle_obj_count(const char* path, uint32_t* n) {
  if (!path || !n) return -1;
  return obj_read(path, NULL, NULL, NULL, 0, n);
}

int oracle_obj_load(const char* path, float* positions, double* normals, double* uvs, uint32_t n) {
  if (!path || !positions || !normals) return -1;
  uint32_t got = 0;
  int rc = obj_read(path, positions, normals, uvs, n, &got);
  if (rc) return rc;
  return got == n ? 0 : -1;
}
