// Host code under AddressSanitizer / UndefinedBehaviorSanitizer:
// rt_scene_parse / rt_scene_load / rt_scene_format (psrt_scenefile.cpp), the
// scene helpers (psrt_scene.cpp) and the culling build (psrt_bvh.cpp) over
// the committed scene files, random scenes and a mutation fuzz of the scene
// text. Built by tests/test_sanitizers.py with -fsanitize=address,undefined
// -fno-sanitize-recover=all, so any report aborts the run.
//
//   scenefile_fuzz <scene files...>     prints "ok <parsed> <rejected>"
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "../../petershirleyraytracer_amd/csrc/psrt_bvh.h"
#include "../../petershirleyraytracer_amd/csrc/psrt_error.h"

// The C ABI's error slot lives in psrt_capi.hip (a HIP source); the host-only
// build needs its own.
namespace psrt {
static thread_local std::string g_msg;
int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_msg = buf;
  return code;
}
}  // namespace psrt

static int fails = 0;
#define CHECK(c, what)                                   \
  do {                                                   \
    if (!(c)) {                                          \
      std::printf("FAIL %s (line %d)\n", what, __LINE__); \
      ++fails;                                           \
    }                                                    \
  } while (0)

// %.17g / strtod keep every finite value and infinity bit for bit; a NaN
// reads back as a NaN (its payload is not part of the text form)
static bool same_bits(double a, double b) {
  return std::memcmp(&a, &b, sizeof a) == 0 || (std::isnan(a) && std::isnan(b));
}

// parse (size query, then fill); on success: format -> parse reproduces every
// bit; the culling build runs over the result. Returns the parse result.
static int parse_roundtrip(const std::string& text) {
  rt_camera cam{};
  // the caller's defaults for keys the file leaves out (valid values, so the
  // formatted render line parses back)
  rt_params p{};
  p.width = 64, p.height = 48, p.spp = 1, p.max_depth = 50;
  const int n = rt_scene_parse(text.c_str(), nullptr, 0, &cam, &p);
  if (n < 0) {
    CHECK(n == RT_E_SCENE || n == RT_E_INVALID, "error code");
    return n;
  }
  std::vector<rt_sphere> s((size_t)n + 1);
  rt_params p2{};
  p2.width = 64, p2.height = 48, p2.spp = 1, p2.max_depth = 50;
  const int n2 = rt_scene_parse(text.c_str(), s.data(), n, nullptr, &p2);
  CHECK(n2 == n, "second parse count");
  s.resize(n);
  const long long len = rt_scene_format(s.data(), n, &cam, &p, nullptr, 0);
  CHECK(len > 0, "format length");
  std::vector<char> buf((size_t)len + 1);
  CHECK(rt_scene_format(s.data(), n, &cam, &p, buf.data(), buf.size()) == len, "format");
  // truncated output stays NUL-terminated
  char small[7];
  rt_scene_format(s.data(), n, &cam, &p, small, sizeof small);
  CHECK(std::strlen(small) == sizeof small - 1, "truncated format");
  std::vector<rt_sphere> back((size_t)n + 1);
  rt_camera cam2{};
  rt_params p3{};
  const int n3 = rt_scene_parse(buf.data(), back.data(), n, &cam2, &p3);
  CHECK(n3 == n, "round-trip count");
  for (int k = 0; k < n && k < n3; ++k)
    CHECK(same_bits(back[k].cx, s[k].cx) && same_bits(back[k].cy, s[k].cy) &&
              same_bits(back[k].cz, s[k].cz) && same_bits(back[k].r, s[k].r),
          "round-trip sphere bits");
  for (int k = 0; k < 3; ++k)
    CHECK(same_bits(cam2.origin[k], cam.origin[k]) && same_bits(cam2.vertical[k], cam.vertical[k]),
          "round-trip camera bits");
  CHECK(p3.width == p.width && p3.height == p.height && p3.spp == p.spp &&
            p3.max_depth == p.max_depth && p3.seed == p.seed,
        "round-trip render line");
  if (n > 0 && n <= 4096) (void)psrt::build_bvh(s.data(), n);  // any scene a file can hold
  return n;
}

static std::string read_file(const char* path) {
  std::string t;
  if (FILE* f = std::fopen(path, "rb")) {
    char b[4096];
    size_t g;
    while ((g = std::fread(b, 1, sizeof b, f)) > 0) t.append(b, g);
    std::fclose(f);
  }
  return t;
}

static const char* kTokens[] = {
    "sphere", "camera", "render", "default", "basis", "look_at", "auto", "width", "height",
    "spp", "depth", "seed", "psrt-scene", "1", "0", "-1", "nan", "inf", "-inf", "0x1p-1074",
    "1e308", "1e309", "-0", "0x", "#", "\n", "\r\n", " ", "\t", "18446744073709551615",
    "18446744073709551616", "9223372036854775808", "1048577", "2147483648", "1e-320", "."};

int main(int argc, char** argv) {
  int parsed = 0, rejected = 0;
  std::vector<std::string> corpus;
  for (int a = 1; a < argc; ++a) {
    corpus.push_back(read_file(argv[a]));
    // rt_scene_load over the real file as well
    const int n = rt_scene_load(argv[a], nullptr, 0, nullptr, nullptr);
    CHECK(n > 0, "committed scene file loads");
  }
  CHECK(rt_scene_load("/nonexistent/scene", nullptr, 0, nullptr, nullptr) == RT_E_INVALID,
        "missing file");
  CHECK(rt_scene_parse(nullptr, nullptr, 0, nullptr, nullptr) == RT_E_INVALID, "null text");
  CHECK(rt_scene_parse("psrt-scene 1\n", nullptr, -1, nullptr, nullptr) == RT_E_INVALID, "cap < 0");
  // random scenes through format -> parse
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> U(-1e3, 1e3);
  for (int t = 0; t < 40; ++t) {
    std::vector<rt_sphere> s(1 + rng() % 300);
    for (auto& q : s) q = {U(rng), U(rng), U(rng), U(rng) * 1e-3};
    if (t % 5 == 0) s[0] = {0.0, -0.0, 0x1p-1074, -1e300};
    rt_camera cam;
    rt_camera_default(&cam);
    const long long len = rt_scene_format(s.data(), (int)s.size(), &cam, nullptr, nullptr, 0);
    std::vector<char> buf((size_t)len + 1);
    rt_scene_format(s.data(), (int)s.size(), &cam, nullptr, buf.data(), buf.size());
    corpus.emplace_back(buf.data());
    CHECK(parse_roundtrip(corpus.back()) == (int)s.size(), "random scene round trip");
  }
  // the final scene of the C ABI helper, with a look-at camera line
  {
    std::vector<rt_sphere> fin(1024);
    const int nf = rt_scene_random_spheres(1, fin.data(), (int)fin.size());
    std::string t = "psrt-scene 1\ncamera look_at 13 2 3 0 0 0 0 1 0 20 auto\n"
                    "render width 1200 height 800 spp 100 depth 50 seed 0\n";
    char line[160];
    for (int k = 0; k < nf; ++k) {
      std::snprintf(line, sizeof line, "sphere %a %a %a %a\n", fin[k].cx, fin[k].cy, fin[k].cz,
                    fin[k].r);
      t += line;
    }
    corpus.push_back(t);
    CHECK(parse_roundtrip(t) == nf, "final scene round trip");
  }
  // the book's scene with materials and the lens camera (host helpers of the
  // materials extension): NULL outputs, truncating caps, degenerate lenses
  {
    const int nb = rt_scene_book_final(1, nullptr, nullptr, 0);
    CHECK(nb == 487, "book scene count");
    std::vector<rt_sphere> bs((size_t)nb);
    std::vector<rt_material> bm((size_t)nb);
    CHECK(rt_scene_book_final(1, bs.data(), bm.data(), nb) == nb, "book scene");
    CHECK(rt_scene_book_final(7, bs.data(), nullptr, 10) == rt_scene_book_final(7, nullptr, nullptr, 0),
          "book scene truncated");
    for (int k = 0; k < nb; ++k)
      CHECK(bm[k].kind >= RT_MAT_LAMBERTIAN && bm[k].kind <= RT_MAT_DIELECTRIC, "material kind");
    const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    rt_camera_lens lc{};
    CHECK(rt_camera_look_at_lens(from, at, up, 20.0, 1.5, 0.1, 10.0, &lc) == RT_OK, "lens camera");
    CHECK(rt_camera_look_at_lens(from, at, up, 20.0, 1.5, -1.0, 10.0, &lc) == RT_E_INVALID,
          "negative aperture");
    CHECK(rt_camera_look_at_lens(from, at, up, 20.0, 1.5, 0.1, 0.0, &lc) == RT_E_INVALID,
          "zero focus distance");
    (void)rt_camera_look_at_lens(from, from, up, 20.0, 1.5, 0.1, 1.0, &lc);  // lookfrom == lookat
  }
  // mutation fuzz: byte flips, deletions, insertions of grammar tokens and
  // random bytes, truncation, duplication of lines
  const int iters = 6000;
  for (int it = 0; it < iters; ++it) {
    std::string t = corpus[rng() % corpus.size()];
    if (t.size() > 4000) t.resize(rng() % 4000);  // keep iterations cheap
    const int muts = 1 + (int)(rng() % 8);
    for (int m = 0; m < muts; ++m) {
      const size_t pos = t.empty() ? 0 : rng() % (t.size() + 1);
      switch (rng() % 6) {
        case 0:
          if (!t.empty() && pos < t.size()) t[pos] = (char)(rng() % 256);
          break;
        case 1:
          if (pos < t.size()) t.erase(pos, 1 + rng() % 16);
          break;
        case 2:
          t.insert(pos, kTokens[rng() % (sizeof kTokens / sizeof kTokens[0])]);
          break;
        case 3:
          t.insert(pos, 1, (char)(1 + rng() % 255));  // never NUL: the text is a C string
          break;
        case 4:
          t.resize(pos);
          break;
        default: {
          const size_t e = t.find('\n', pos);
          if (e != std::string::npos) t.insert(pos, t.substr(pos, e - pos + 1));
        }
      }
    }
    t.erase(std::remove(t.begin(), t.end(), '\0'), t.end());
    if (parse_roundtrip(t) >= 0)
      ++parsed;
    else
      ++rejected;
  }
  // a very long line and deep number lists
  parse_roundtrip("psrt-scene 1\nsphere " + std::string(100000, '1') + " 0 0 1\n");
  parse_roundtrip("psrt-scene 1\nrender " + std::string(20000, ' ') + "spp 4\n");
  std::printf("ok %d %d\n", parsed, rejected);
  return fails ? 1 : 0;
}
