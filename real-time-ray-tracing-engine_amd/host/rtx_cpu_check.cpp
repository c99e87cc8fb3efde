// rtx_cpu_check — host-only driver of the CPU backend (host/rtx_cpu.cpp) for
// the sanitizer builds (make sanitize: TSan over its row pool, ASan/UBSan over
// the per-path code): loads each scene file, sets up its camera at a small
// size and renders it with rt_cpu_render on --threads N, twice; the two
// frames must be equal bit for bit (a pixel's strata are summed in stratum
// order on one thread whatever the thread count).  Exit status 0 when every
// scene renders and repeats, 1 otherwise.
//
//   rtx_cpu_check [--threads N] [--width W] [--spp S] file.json...
#include "rt_cpu.h"
#include "scene_json.hpp"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace rtx {
int camera_setup(const rt_camera_desc *cd, rt_frame *f, std::string &err);
}

int main(int argc, char **argv) {
  int threads = 8, width = 48, spp = 9;
  std::vector<std::string> files;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) threads = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--width") && i + 1 < argc) width = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--spp") && i + 1 < argc) spp = std::atoi(argv[++i]);
    else files.push_back(argv[i]);
  }
  if (files.empty()) {
    std::fprintf(stderr, "usage: rtx_cpu_check [--threads N] [--width W] [--spp S] file.json...\n");
    return 2;
  }
  int bad = 0;
  for (const std::string &path : files) {
    rtxhost::LoadedScene S;
    try {
      S = rtxhost::load_scene_file(path);
    } catch (const std::exception &e) {
      std::fprintf(stderr, "%s: %s\n", path.c_str(), e.what());
      ++bad;
      continue;
    }
    rt_camera_desc cam = S.camera;
    cam.image_width = width;
    cam.samples_per_pixel = spp;
    cam.max_depth = 8;
    rt_frame f;
    std::string err;
    if (rtx::camera_setup(&cam, &f, err) != RT_OK) {
      std::fprintf(stderr, "%s: camera: %s\n", path.c_str(), err.c_str());
      ++bad;
      continue;
    }
    rt_scene_desc d = S.desc();
    rt_render_params p{};
    p.sample_count = -1;
    p.seed = 3;
    p.output = RT_OUT_SUM;
    std::vector<double> a((size_t)f.image_width * f.image_height * 3), b(a.size());
    if (rt_cpu_render(&d, &f, &p, threads, a.data()) != RT_OK ||
        rt_cpu_render(&d, &f, &p, threads, b.data()) != RT_OK) {
      std::fprintf(stderr, "%s: render: %s\n", path.c_str(), rt_cpu_last_error());
      ++bad;
      continue;
    }
    const bool same = std::memcmp(a.data(), b.data(), a.size() * sizeof(double)) == 0;
    double sum = 0;
    for (double x : a) sum += x;
    std::printf("%s: %dx%d spp %d, %d threads, sum %.17g, repeat %s\n", path.c_str(), f.image_width,
                f.image_height, f.sqrt_spp * f.sqrt_spp, threads, sum, same ? "bit-identical" : "DIFFERS");
    if (!same) ++bad;
  }
  return bad ? 1 : 0;
}
