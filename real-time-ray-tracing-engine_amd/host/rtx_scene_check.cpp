// rtx_scene_check — validates JSON scene files on the host, without a GPU.
//
// Runs the two host stages every render goes through before any device call:
// the JSON loader (host/json_min.hpp + host/scene_json.hpp, what rtx_render
// uses) and the library's scene compiler (csrc/rt_scene.cpp: flattening,
// validation, BVH build, light leaves -- the work initialize_cuda_scene and the
// converters do in the reference, CudaSceneInitialization.cuh:249-300), plus
// the camera setup (Camera::initialize, Camera.cpp:31-73).  Prints one line per
// file; exit status 0 = all valid, 1 = a file was rejected with a message.
//
//   rtx_scene_check [--threads N] [--repeat K] file.json...
//
// --threads N compiles every file from N host threads at once (K times each):
// the library's contract is that distinct scenes are built and used from
// different host threads independently (rt_api.h "Threading"); the TSan build
// of this tool (make sanitize) checks that the host stages share no state.
#include "../csrc/rt_scene.h"
#include "scene_json.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct Result {
  bool ok = false;
  std::string msg;
};

Result check_file(const std::string &path) {
  Result r;
  try {
    rtxhost::LoadedScene S = rtxhost::load_scene_file(path);
    rt_scene_desc d = S.desc();
    rtx::HostScene H;
    std::string err;
    int rc = rtx::compile_scene(&d, H, err);
    if (rc != RT_OK) {
      r.msg = "scene: " + err;
      return r;
    }
    if (H.device_bvh) rtx::build_world_bvh_host(H); // the host twin of the device build
    rt_frame f;
    if (rtx::camera_setup(&S.camera, &f, err) != RT_OK) {
      r.msg = "camera: " + err;
      return r;
    }
    char b[256];
    std::snprintf(b, sizeof b, "%d items, %d media, %d nodes (depth %d), %d lights, %dx%d",
                  (int)H.items.size(), (int)H.mitems.size(), (int)H.nodes.size(), H.bvh_depth,
                  (int)H.lights.size(), f.image_width, f.image_height);
    r.ok = true;
    r.msg = b;
  } catch (const std::exception &e) {
    r.msg = e.what();
  }
  return r;
}

} // namespace

int main(int argc, char **argv) {
  int threads = 1, repeat = 1;
  std::vector<std::string> files;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--threads") && i + 1 < argc)
      threads = std::max(1, std::atoi(argv[++i]));
    else if (!std::strcmp(argv[i], "--repeat") && i + 1 < argc)
      repeat = std::max(1, std::atoi(argv[++i]));
    else
      files.push_back(argv[i]);
  }
  if (files.empty()) {
    std::fprintf(stderr, "usage: rtx_scene_check [--threads N] [--repeat K] file.json...\n");
    return 2;
  }
  // every thread checks every file `repeat` times; all threads must agree
  std::vector<std::vector<Result>> per(threads, std::vector<Result>(files.size()));
  auto work = [&](int t) {
    for (int rep = 0; rep < repeat; ++rep)
      for (size_t n = 0; n < files.size(); ++n) {
        size_t k = (n + t) % files.size(); // threads start on different files
        per[t][k] = check_file(files[k]);
      }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto &th : pool) th.join();
  const std::vector<Result> &res = per[0];
  for (int t = 1; t < threads; ++t)
    for (size_t k = 0; k < files.size(); ++k)
      if (per[t][k].ok != res[k].ok || per[t][k].msg != res[k].msg) {
        std::fprintf(stderr, "thread %d disagrees on %s\n", t, files[k].c_str());
        return 3;
      }
  int rc = 0;
  for (size_t k = 0; k < files.size(); ++k) {
    std::printf("%s: %s %s\n", files[k].c_str(), res[k].ok ? "ok" : "REJECTED", res[k].msg.c_str());
    if (!res[k].ok) rc = 1;
  }
  return rc;
}
