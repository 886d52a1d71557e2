// psrt::pinned_frame (page-locked host buffers, rt_host_alloc) against the
// ordinary frame: the same bits through rt_render and rt_group_render, a
// pinned frame reused for a second render, and a bytes-only frame
// (want_accum = false) (tests/test_host_api.py).
#include <cstdio>
#include <cstring>
#include <vector>

#include "psrt/render.hpp"

template <class A, class B>
static bool same(const A& a, const B& b) {
  return a.size() == b.size() && std::memcmp(a.data(), b.data(), a.size() * sizeof(a[0])) == 0;
}

int main() {
  const int n = rt_scene_random_spheres(1, nullptr, 0);
  std::vector<rt_sphere> sph((size_t)n);
  rt_scene_random_spheres(1, sph.data(), n);
  const double from[3] = {13, 2, 3}, at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
  rt_camera c{};
  psrt::check(rt_camera_look_at(from, at, up, 20.0, 96.0 / 64.0, &c), "look_at");
  const hittable_list world = psrt::to_world(sph);
  const camera cam = psrt::to_camera(c);
  const psrt::frame want = psrt::render(world, cam, 96, 64, 8, 50, 5);
  psrt::pinned_frame pf;
  psrt::render_into(pf, world, cam, 96, 64, 8, 50, 5);
  const void* keep = pf.accum.data();
  if (!same(pf.accum, want.accum) || !same(pf.rgb8, want.rgb8)) return std::puts("pinned differs"), 1;
  // reused (no reallocation): another seed, then the first again
  psrt::render_into(pf, world, cam, 96, 64, 8, 50, 6);
  if (pf.accum.data() != keep) return std::puts("reallocated"), 1;
  if (same(pf.accum, want.accum)) return std::puts("seed ignored"), 1;
  psrt::render_into(pf, world, cam, 96, 64, 8, 50, 5);
  if (!same(pf.accum, want.accum) || !same(pf.rgb8, want.rgb8)) return std::puts("reuse differs"), 1;
  // a 1:3 shard into a pinned frame, and three group members into one
  const psrt::frame shard = psrt::render(world, cam, 96, 64, 8, 50, 5, 1, 3);
  psrt::render_into(pf, world, cam, 96, 64, 8, 50, 5, 1, 3);
  if (!same(pf.accum, shard.accum) || pf.rows != shard.rows) return std::puts("shard differs"), 1;
  psrt::device_group g({0, 0, 0});
  g.set_scene(world, cam);
  psrt::pinned_frame gf;
  g.render_into(gf, 96, 64, 8, 50, 5);
  if (!same(gf.accum, want.accum) || !same(gf.rgb8, want.rgb8)) return std::puts("group differs"), 1;
  // the bytes alone (what main.cc prints): the sums stay on the device
  psrt::pinned_frame bf;
  bf.want_accum = false;
  psrt::render_into(bf, world, cam, 96, 64, 8, 50, 5);
  if (!bf.accum.empty() || !same(bf.rgb8, want.rgb8)) return std::puts("bytes-only differs"), 1;
  std::puts("ok");
  return 0;
}
