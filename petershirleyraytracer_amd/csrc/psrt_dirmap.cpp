// psrt_dirmap.cpp — host plan of the direction maps (psrt_dirmap.h).
//
// The bits themselves are computed on the device (psrt_dir_maps): for every
// map, every BVH sphere against every direction bin. Here: the patches, their
// origin balls (conservative, FP64) and the bin cones.
#include "psrt_dirmap.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

namespace psrt {
namespace {

// The vector of cube cell coordinates (s, t) on face f (psrt_dirmap.h).
void face_vec(int f, double s, double t, double v[3]) {
  const int m = f >> 1, u = m == 0 ? 1 : 0, w = m == 2 ? 1 : 2;
  v[m] = (f & 1) ? -1.0 : 1.0;
  v[u] = s;
  v[w] = t;
}

double angle(const double a[3], const double b[3]) {
  const double cx = a[1] * b[2] - a[2] * b[1], cy = a[2] * b[0] - a[0] * b[2],
               cz = a[0] * b[1] - a[1] * b[0];
  return std::atan2(std::sqrt(cx * cx + cy * cy + cz * cz), a[0] * b[0] + a[1] * b[1] + a[2] * b[2]);
}

// Unit axis and half-angle of a cone holding every direction of cube cell
// (i, j) of an M x M face f, the cell widened by kDirEps: the angle to a fixed
// axis is quasi-convex on the face plane (its sublevel sets are conic
// sections' convex sides), so its maximum over the cell is at a corner.
void cell_cone(int f, int M, int i, int j, double axis[3], double* half) {
  const double s0 = -1.0 + 2.0 * i / M - kDirEps, s1 = -1.0 + 2.0 * (i + 1) / M + kDirEps;
  const double t0 = -1.0 + 2.0 * j / M - kDirEps, t1 = -1.0 + 2.0 * (j + 1) / M + kDirEps;
  face_vec(f, 0.5 * (s0 + s1), 0.5 * (t0 + t1), axis);
  const double l = std::sqrt(axis[0] * axis[0] + axis[1] * axis[1] + axis[2] * axis[2]);
  for (int k = 0; k < 3; ++k) axis[k] /= l;
  double h = 0.0;
  const double ss[2] = {s0, s1}, ts[2] = {t0, t1};
  for (int c = 0; c < 4; ++c) {
    double v[3];
    face_vec(f, ss[c & 1], ts[c >> 1], v);
    h = std::max(h, angle(axis, v));
  }
  *half = h + 1e-9;
}

}  // namespace

DirMapHost plan_dirmaps(const rt_sphere* s, int n, const BvhHost& b) {
  DirMapHost out;
  if (!b.enabled || n <= 0 || std::getenv("PSRT_NO_DIRMAP")) return out;
  // patch edge: PSRT_DIRMAP_H median radii (tuning knob, default 0.35)
  std::vector<double> radii(n);
  for (int k = 0; k < n; ++k) radii[k] = std::fabs(s[k].r);
  std::vector<double> sorted = radii;
  std::nth_element(sorted.begin(), sorted.begin() + n / 2, sorted.end());
  const char* eh = std::getenv("PSRT_DIRMAP_H");
  double h = (eh ? std::atof(eh) : 0.35) * sorted[n / 2];
  if (!(h > 0.0)) return out;
  const char* em = std::getenv("PSRT_DIRMAP_MAX");
  const long max_maps = em ? std::atol(em) : (1L << 20);
  std::vector<char> is_big(n, 0);
  for (int k : b.big_idx) is_big[k] = 1;
  // big spheres: the part of the surface whose rays start near the BVH spheres
  // (the grid box widened by 4 patch edges)
  double blo[3], bhi[3];
  for (int k = 0; k < 3; ++k) {
    blo[k] = (double)b.grid.flo[k];
    bhi[k] = (double)b.grid.fhi[k];
  }
  const double kHalfPi = 1.5707963267948966;
  for (int attempt = 0; attempt < 16; ++attempt, h *= 1.5) {
    out.desc.assign((size_t)n * 6 * 4, 0);
    long maps = 0;
    for (int k = 0; k < n; ++k) {
      const double R = radii[k];
      for (int f = 0; f < 6; ++f) out.desc[(k * 6 + f) * 4] = -1;
      if (!(R > 4.0 * b.pad)) continue;  // too small for a patch ball inside the pad budget
      const int M = (int)std::min<double>(kDirMaxM, std::max(1.0, std::ceil(kHalfPi * R / h)));
      const double c[3] = {s[k].cx, s[k].cy, s[k].cz};
      for (int f = 0; f < 6; ++f) {
        int i0 = 0, j0 = 0, ni = M, nj = M;
        if (is_big[k]) {
          const int m = f >> 1, u = m == 0 ? 1 : 0, w = m == 2 ? 1 : 2;
          const double sg = (f & 1) ? -1.0 : 1.0;
          double smin = 1e300, smax = -1e300, tmin = 1e300, tmax = -1e300;
          bool ok = true;
          for (int q = 0; q < 8; ++q) {
            const double g = 4.0 * h;
            const double p[3] = {(q & 1) ? bhi[0] + g : blo[0] - g, (q & 2) ? bhi[1] + g : blo[1] - g,
                                 (q & 4) ? bhi[2] + g : blo[2] - g};
            const double dm = sg * (p[m] - c[m]);
            if (!(dm > 0.0)) {
              ok = false;
              break;
            }
            const double ss = (p[u] - c[u]) / dm, tt = (p[w] - c[w]) / dm;
            smin = std::min(smin, ss), smax = std::max(smax, ss);
            tmin = std::min(tmin, tt), tmax = std::max(tmax, tt);
          }
          if (!ok || smax < -1.0 || smin > 1.0 || tmax < -1.0 || tmin > 1.0) continue;
          auto cl = [M](double x) { return (int)std::max(0.0, std::min((double)(M - 1), x)); };
          i0 = cl(std::floor((smin + 1.0) * 0.5 * M) - 1.0);
          const int i1 = cl(std::floor((smax + 1.0) * 0.5 * M) + 1.0);
          j0 = cl(std::floor((tmin + 1.0) * 0.5 * M) - 1.0);
          const int j1 = cl(std::floor((tmax + 1.0) * 0.5 * M) + 1.0);
          ni = i1 - i0 + 1;
          nj = j1 - j0 + 1;
        }
        int32_t* d = &out.desc[(k * 6 + f) * 4];
        d[0] = (int32_t)maps;
        d[1] = M;
        d[2] = (int32_t)((uint32_t)i0 | (uint32_t)j0 << 16);
        d[3] = (int32_t)((uint32_t)ni | (uint32_t)nj << 16);
        maps += (long)ni * nj;
      }
    }
    if (maps > max_maps) continue;  // coarser patches
    out.n_maps = (int)maps;
    out.h = h;
    break;
  }
  if (out.h == 0.0) {  // no budget: no maps
    out.desc.clear();
    return out;
  }
  // origin balls: o within pad/2 of the surface (the device checks
  // C^2 <= (pad/2)^2 r^2, so ||o - c| - r| <= pad/2) and (o - c) in the widened
  // patch cone (axis a, half-angle beta): |o - (c + r a)| <= pad/2 + r beta.
  // Radius: r beta + pad (a 2x margin on the radial part).
  out.ball.resize((size_t)out.n_maps * 4);
  out.excl.resize(out.n_maps);
  for (int k = 0; k < n; ++k) {
    for (int f = 0; f < 6; ++f) {
      const int32_t* d = &out.desc[(k * 6 + f) * 4];
      if (d[0] < 0) continue;
      const int M = d[1], i0 = d[2] & 0xFFFF, j0 = (int)((uint32_t)d[2] >> 16), ni = d[3] & 0xFFFF,
                nj = (int)((uint32_t)d[3] >> 16);
      for (int i = 0; i < ni; ++i)
        for (int j = 0; j < nj; ++j) {
          double a[3], beta;
          cell_cone(f, M, i0 + i, j0 + j, a, &beta);
          const long mi = (long)d[0] + (long)i * nj + j;
          double* bl = &out.ball[mi * 4];
          bl[0] = s[k].cx + radii[k] * a[0];
          bl[1] = s[k].cy + radii[k] * a[1];
          bl[2] = s[k].cz + radii[k] * a[2];
          bl[3] = (radii[k] * (beta + 1e-12) + b.pad) * (1.0 + 0x1p-40);
          out.excl[mi] = is_big[k] ? -1 : k;
        }
    }
  }
  // direction bins
  out.bins.assign((size_t)kDirBins * 8, 0.0);
  for (int f = 0; f < 6; ++f)
    for (int i = 0; i < kDirN; ++i)
      for (int j = 0; j < kDirN; ++j) {
        double a[3], ha;
        cell_cone(f, kDirN, i, j, a, &ha);
        double* e = &out.bins[(size_t)((f * kDirN + i) * kDirN + j) * 8];
        e[0] = a[0], e[1] = a[1], e[2] = a[2];
        e[3] = std::cos(ha);
        e[4] = std::sin(ha);
      }
  return out;
}

}  // namespace psrt
