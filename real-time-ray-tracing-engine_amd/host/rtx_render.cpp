// rtx_render — command-line front end over librtx_hip.so (include/rt_api.h).
//
// Takes the reference binary's flags (input/CLI.cpp:4-95, same names, defaults
// and messages) plus a JSON scene, renders the static camera's frame on the
// GPU through the C ABI and writes output/<file> as a P3 PPM with write_color's
// quantisation (StaticCamera.cpp:50-57, ColorUtility.hpp:11-36).
//
//   rtx_render [--camera static] [--output image.ppm] [-p] [-b] [-g] [-d]
//              [--width N] [--samples N] [--depth N]
//              [--scene file.json] [--seed S] [--device D] [--gpus N] [--shards K]
//              [--backend hip|cpu] [--threads N] [--dump-desc]
//
// Mapping of the reference flags onto this library:
//   --camera static   the only mode; "dynamic" is the SDL window (out of scope,
//                     DESIGN.md) and is rejected with a message.
//   -p / -g           accepted; the backend is --backend's (default hip: the GPU
//                     library).  The reference's -p without -g selects its CPU
//                     path; here that is --backend cpu.
//   --backend cpu     the CPU backend (librtx_cpu.so, include/rt_cpu.h): the
//                     kernel's per-path source compiled for the host, image rows
//                     on --threads N host threads (default: the CPUs this
//                     process may use -- affinity mask and cgroup quota,
//                     rt_cpu_default_threads; StaticCamera::render_cpu's ThreadPool role,
//                     StaticCamera.cpp:32-134).  Chosen, never a fallback: the
//                     default backend fails if the GPU library cannot render.
//   -b                scene use_bvh (the reference's light-list BVH split); the
//                     world BVH is always built on the device.
//   -d                writes the flattened scene description to logs/scene_desc.json
//                     (the reference writes its scene JSON to logs/, Camera.cpp:82).
//   --width/--samples/--depth
//                     reference defaults 600/100/50 when --scene is not given
//                     (main.cpp:150-156 always uses them); with --scene the file's
//                     camera block is the default and the flags override it.
// Extensions: --scene (default scenes/cornell.json next to the library, the
// reference's default populate_cornell_box_scene), --seed (the Philox key that
// replaces curand_init(time(nullptr)+pixel)), --device, --dump-desc (print the
// description as JSON and exit; used by tests/test_cli.py), and the multi-GPU
// flags SURVEY §5 adds: --gpus N renders on devices device..device+N-1 through
// rt_multi_* (one host thread and one scene per shard, 8x8 tiles dealt
// round-robin; each shard sums its chunk partials on its own device, its tiles
// are peer-copied to the first shard's device -- xGMI between GPUs -- and
// reordered into the frame there, one D2H copy per frame: rt_api.cpp
// rt_multi_render); --shards K (default N) splits
// the frame into K tile shards, K > N putting several shards on one device.
// The sharded frame is bit-identical to the one-device frame (rt_api.h).
#include "rt_api.h"
#include "rt_cpu.h"
#include "scene_json.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>
#include <sys/stat.h>
#include <vector>

namespace {

struct Options {
  int width = 600, samples = 100, depth = 50; // CLI.hpp:11-13
  bool width_set = false, samples_set = false, depth_set = false;
  bool help = false, use_static = true, parallel = false, use_bvh = false, gpu = false;
  bool any_errors = false, debug = false, dump_desc = false;
  std::string output = "image.ppm";
  std::string scene;
  unsigned long long seed = 0;
  int device = 0;
  int gpus = 1, shards = 0;
  bool cpu = false; // --backend cpu
  int threads = 0;  // --threads (CPU backend); 0: rt_cpu_default_threads()
};

bool parse_int(const char *s, int &out) {
  try {
    out = std::stoi(s);
    return true;
  } catch (...) {
    return false;
  }
}

Options parse(int argc, char **argv) {
  Options o;
  bool output_selected = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto need = [&](const char *what) -> const char * {
      if (i + 1 < argc) return argv[++i];
      o.any_errors = true;
      std::cerr << a << " requires " << what << "\n";
      return nullptr;
    };
    if (a == "-h" || a == "--help") {
      o.help = true;
    } else if (a == "--camera") {
      if (const char *t = need("an argument: static or dynamic")) {
        std::string ty = t;
        if (ty == "static") o.use_static = true;
        else if (ty == "dynamic") o.use_static = false;
        else {
          o.any_errors = true;
          std::cerr << "Unknown camera type: " << ty << std::endl;
        }
      }
    } else if (a == "--output") {
      if (const char *f = need("a filename")) {
        o.output = f;
        output_selected = true;
      }
    } else if (a == "-p" || a == "--parallel") {
      o.parallel = true;
    } else if (a == "-b" || a == "--bvh") {
      o.use_bvh = true;
    } else if (a == "-g" || a == "--gpu") {
      o.gpu = true;
    } else if (a == "-d" || a == "--debug") {
      o.debug = true;
    } else if (a == "--backend") {
      if (const char *b = need("an argument: hip or cpu")) {
        std::string be = b;
        if (be == "hip" || be == "gpu") o.cpu = false;
        else if (be == "cpu") o.cpu = true;
        else {
          o.any_errors = true;
          std::cerr << "Unknown backend: " << be << " (hip or cpu)\n";
        }
      }
    } else if (a == "--width" || a == "--samples" || a == "--depth" || a == "--device" ||
               a == "--gpus" || a == "--shards" || a == "--threads") {
      if (const char *v = need("a number")) {
        int x;
        if (!parse_int(v, x)) {
          o.any_errors = true;
          std::cerr << a << " requires a valid integer\n";
        } else if (a == "--width") {
          o.width = x;
          o.width_set = true;
        } else if (a == "--samples") {
          o.samples = x;
          o.samples_set = true;
        } else if (a == "--depth") {
          o.depth = x;
          o.depth_set = true;
        } else if (a == "--gpus") {
          o.gpus = x;
        } else if (a == "--shards") {
          o.shards = x;
        } else if (a == "--threads") {
          o.threads = x;
        } else {
          o.device = x;
        }
      }
    } else if (a == "--scene") {
      if (const char *f = need("a scene file")) o.scene = f;
    } else if (a == "--seed") {
      if (const char *v = need("a number")) o.seed = std::strtoull(v, nullptr, 0);
    } else if (a == "--dump-desc") {
      o.dump_desc = true;
    } else {
      o.any_errors = true;
      std::cerr << "Unknown option: " << a << std::endl;
    }
  }
  if (o.gpus < 1 || o.shards < 0 || (o.shards && o.shards < o.gpus)) {
    o.any_errors = true;
    std::cerr << "--gpus must be >= 1 and --shards >= --gpus\n";
  }
  if (o.threads < 0) {
    o.any_errors = true;
    std::cerr << "--threads must be >= 0\n";
  }
  if (o.cpu && (o.gpus > 1 || o.shards > 1)) {
    o.any_errors = true;
    std::cerr << "--gpus / --shards are GPU options; --backend cpu uses --threads\n";
  }
  if (!o.use_static && output_selected)
    std::cerr << "You can only set an output file if the static camera is selected, ignoring...\n";
  return o;
}

void print_help() {
  std::cout
      << "rtx_render: path-traced still frames on MI355X through librtx_hip.\n\n"
         "Usage: rtx_render [options]\n\n"
         "Options:\n"
         "  -h, --help                 Show this help message\n"
         "  --camera [static|dynamic]  Camera type (default: static; dynamic is not provided)\n"
         "  --output <file>            Output file under output/ (default: image.ppm)\n"
         "  -p, --parallel             Accepted (both backends are parallel)\n"
         "  -b, --bvh                  Use the reference's BVH light-list split (use_bvh)\n"
         "  -g, --gpu                  Accepted (the default backend is the GPU)\n"
         "  -d, --debug                Write the scene description to logs/scene_desc.json\n"
         "  --width <int>              Image width (default: 600)\n"
         "  --samples <int>            Samples per pixel (default: 100)\n"
         "  --depth <int>              Maximum bounces (default: 50)\n"
         "  --scene <file.json>        Scene file (default: scenes/cornell.json)\n"
         "  --seed <u64>               Sample-stream key (default: 0)\n"
         "  --device <int>             HIP device ordinal (default: 0)\n"
         "  --gpus <int>               Devices to render on, from --device (default: 1)\n"
         "  --shards <int>             Tile shards over those devices (default: --gpus)\n"
         "  --backend <hip|cpu>        GPU library (default) or the CPU backend\n"
         "  --threads <int>            CPU backend threads (default: the CPUs this process may use)\n"
         "  --dump-desc                Print the flattened scene description and exit\n";
}

std::string exe_dir(const char *argv0) {
  std::string p = argv0;
  size_t s = p.find_last_of('/');
  return s == std::string::npos ? std::string(".") : p.substr(0, s);
}

bool file_exists(const std::string &p) {
  struct stat st;
  return stat(p.c_str(), &st) == 0;
}

// ---- JSON dump of the description (round-trip %.17g) ----------------------
void jv(std::ostream &os, const rt_vec3 &v) {
  char b[96];
  std::snprintf(b, sizeof b, "[%.17g,%.17g,%.17g]", v.x, v.y, v.z);
  os << b;
}
void jd(std::ostream &os, double x) {
  char b[40];
  std::snprintf(b, sizeof b, "%.17g", x);
  os << b;
}

void dump_desc(std::ostream &os, const rtxhost::LoadedScene &S, const rt_camera_desc &c) {
  os << "{\"textures\":[";
  for (size_t k = 0; k < S.textures.size(); ++k) {
    const rt_texture_desc &t = S.textures[k];
    os << (k ? "," : "") << "{\"kind\":" << t.kind << ",\"even\":" << t.even << ",\"odd\":" << t.odd
       << ",\"perlin\":" << t.perlin << ",\"scale\":";
    jd(os, t.scale);
    os << ",\"color\":";
    jv(os, t.color);
    os << "}";
  }
  os << "],\"perlin\":[";
  for (size_t k = 0; k < S.perlin.size(); ++k) {
    const rt_perlin_desc &p = S.perlin[k];
    long long sx = 0, sy = 0, sz = 0;
    double sv = 0;
    for (int i = 0; i < 256; ++i) {
      sx += (long long)p.perm_x[i] * (i + 1);
      sy += (long long)p.perm_y[i] * (i + 1);
      sz += (long long)p.perm_z[i] * (i + 1);
      sv += p.rand_vec[i].x + 2 * p.rand_vec[i].y + 3 * p.rand_vec[i].z;
    }
    os << (k ? "," : "") << "{\"perm_x\":" << sx << ",\"perm_y\":" << sy << ",\"perm_z\":" << sz
       << ",\"rand_vec\":";
    jd(os, sv);
    os << "}";
  }
  os << "],\"materials\":[";
  for (size_t k = 0; k < S.materials.size(); ++k) {
    const rt_material_desc &m = S.materials[k];
    os << (k ? "," : "") << "{\"kind\":" << m.kind << ",\"texture\":" << m.texture << ",\"albedo\":";
    jv(os, m.albedo);
    os << ",\"fuzz\":";
    jd(os, m.fuzz);
    os << ",\"refraction_index\":";
    jd(os, m.refraction_index);
    os << "}";
  }
  os << "],\"objects\":[";
  for (size_t k = 0; k < S.objects.size(); ++k) {
    const rt_object_desc &o = S.objects[k];
    os << (k ? "," : "") << "{\"kind\":" << o.kind << ",\"material\":" << o.material
       << ",\"child\":" << o.child << ",\"count\":" << o.count << ",\"a\":";
    jv(os, o.a);
    os << ",\"b\":";
    jv(os, o.b);
    os << ",\"c\":";
    jv(os, o.c);
    os << ",\"s\":";
    jd(os, o.s);
    os << ",\"moving\":" << o.moving << ",\"phase\":" << o.phase << "}";
  }
  os << "],\"children\":[";
  for (size_t k = 0; k < S.children.size(); ++k) os << (k ? "," : "") << S.children[k];
  os << "],\"world\":" << S.world << ",\"lights\":" << S.lights << ",\"use_bvh\":" << S.use_bvh;
  os << ",\"camera\":{\"image_width\":" << c.image_width << ",\"samples_per_pixel\":"
     << c.samples_per_pixel << ",\"max_depth\":" << c.max_depth << ",\"aspect_ratio\":";
  jd(os, c.aspect_ratio);
  os << ",\"vfov\":";
  jd(os, c.vfov);
  os << ",\"defocus_angle\":";
  jd(os, c.defocus_angle);
  os << ",\"focus_dist\":";
  jd(os, c.focus_dist);
  os << ",\"lookfrom\":";
  jv(os, c.lookfrom);
  os << ",\"lookat\":";
  jv(os, c.lookat);
  os << ",\"vup\":";
  jv(os, c.vup);
  os << ",\"background\":";
  jv(os, c.background);
  os << "}}\n";
}

// write_color (ColorUtility.hpp:11-36): gamma 2 (sqrt of positive values, else
// 0 — NaN lands on 0), clamp to [0, 0.999], scale by 256, truncate.
unsigned char to_byte(double x) {
  double g = x > 0 ? std::sqrt(x) : 0.0;
  if (g < 0.0) g = 0.0;
  if (g > 0.999) g = 0.999;
  return (unsigned char)(256.0 * g);
}

int fail_rt(const char *what) {
  std::cerr << "[ERROR] " << what << ": " << rt_last_error() << "\n";
  return 1;
}

} // namespace

int main(int argc, char **argv) {
  Options opt = parse(argc, argv);
  if (opt.help) {
    print_help();
    return 0;
  }
  if (opt.any_errors) return 2;
  if (!opt.use_static) {
    std::cerr << "The dynamic (SDL window) camera is not provided by this library; "
                 "use --camera static.\n";
    return 2;
  }

  std::string scene_path = opt.scene;
  bool builtin = scene_path.empty();
  if (builtin) {
    std::string d = exe_dir(argv[0]);
    for (const char *cand : {"/../scenes/cornell.json", "/scenes/cornell.json"})
      if (file_exists(d + cand)) {
        scene_path = d + cand;
        break;
      }
    if (scene_path.empty()) {
      std::cerr << "[ERROR] default scene scenes/cornell.json not found; pass --scene\n";
      return 1;
    }
  }

  rtxhost::LoadedScene S;
  try {
    S = rtxhost::load_scene_file(scene_path);
  } catch (const std::exception &e) {
    std::cerr << "[ERROR] " << scene_path << ": " << e.what() << "\n";
    return 1;
  }
  if (opt.use_bvh) S.use_bvh = 1;
  rt_camera_desc cam = S.camera;
  if (builtin || opt.width_set) cam.image_width = opt.width;
  if (builtin || opt.samples_set) cam.samples_per_pixel = opt.samples;
  if (builtin || opt.depth_set) cam.max_depth = opt.depth;

  if (opt.dump_desc || opt.debug) {
    if (opt.dump_desc) {
      dump_desc(std::cout, S, cam);
      return 0;
    }
    mkdir("logs", 0755);
    std::ofstream f("logs/scene_desc.json", std::ios::out | std::ios::trunc);
    dump_desc(f, S, cam);
  }

  if (rt_abi_version() != RT_ABI_VERSION) {
    std::cerr << "[ERROR] librtx_hip ABI version " << rt_abi_version() << ", this host was built for "
              << RT_ABI_VERSION << "\n";
    return 1;
  }
  rt_frame frame;
  if (rt_camera_setup(&cam, &frame) != RT_OK) return fail_rt("camera");
  rt_scene_desc desc = S.desc();
  rt_scene *scene = nullptr;
  rt_multi *multi = nullptr;
  const int shards = opt.shards ? opt.shards : opt.gpus;
  if (opt.cpu) {
    if (rt_cpu_abi_version() != RT_CPU_ABI_VERSION) {
      std::cerr << "[ERROR] librtx_cpu ABI version " << rt_cpu_abi_version() << ", this host was built for "
                << RT_CPU_ABI_VERSION << "\n";
      return 1;
    }
  } else if (shards > 1) {
    int32_t ndev = 0;
    if (rt_device_count(&ndev) != RT_OK) return fail_rt("device count");
    if (opt.device < 0 || opt.device + opt.gpus > ndev) {
      std::cerr << "[ERROR] --device " << opt.device << " --gpus " << opt.gpus << " needs "
                << opt.device + opt.gpus << " devices, " << ndev << " present\n";
      return 1;
    }
    std::vector<int32_t> devs;
    for (int d = 0; d < opt.gpus; ++d) devs.push_back(opt.device + d);
    if (rt_multi_create(&desc, devs.data(), opt.gpus, shards, &multi) != RT_OK)
      return fail_rt("scene");
  } else if (rt_scene_create(&desc, opt.device, &scene) != RT_OK) {
    return fail_rt("scene");
  }
  auto release = [&]() {
    if (scene) rt_scene_destroy(scene);
    if (multi) rt_multi_destroy(multi);
  };

  const int W = frame.image_width, H = frame.image_height;
  const int n_strata = frame.sqrt_spp * frame.sqrt_spp;
  std::vector<double> sum((size_t)W * H * 3, 0.0), part((size_t)W * H * 3);
  // Strata in chunks so progress is visible on long renders (the reference
  // prints scanlines remaining, StaticCamera.cpp:60-62).
  const long long per_chunk = std::max<long long>(1, 64LL * 2073600 / ((long long)W * H));
  auto t0 = std::chrono::steady_clock::now();
  for (int s = 0; s < n_strata; s += (int)per_chunk) {
    int cnt = (int)std::min<long long>(per_chunk, n_strata - s);
    rt_render_params p{};
    p.row_begin = 0;
    p.row_end = 0;
    p.sample_begin = s;
    p.sample_count = cnt;
    p.seed = opt.seed;
    p.output = RT_OUT_SUM;
    if (opt.cpu) {
      if (rt_cpu_render(&desc, &frame, &p, opt.threads, part.data()) != RT_OK) {
        std::cerr << "[ERROR] render: " << rt_cpu_last_error() << "\n";
        return 1;
      }
    } else if ((multi ? rt_multi_render(multi, &frame, &p, part.data())
                      : rt_render(scene, &frame, &p, part.data())) != RT_OK) {
      int rc = fail_rt("render");
      release();
      return rc;
    }
    for (size_t k = 0; k < sum.size(); ++k) sum[k] += part[k];
    std::clog << "\rStrata remaining: " << (n_strata - s - cnt) << ' ' << std::flush;
  }
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  release();
  std::clog << "\rDone. " << W << "x" << H << " @ " << n_strata << " spp, "
            << (double)W * H * n_strata / secs / 1e6 << " Msamples/s";
  if (opt.cpu)
    std::clog << " (CPU backend, " << (opt.threads > 0 ? opt.threads : rt_cpu_default_threads()) << " threads)";
  else if (shards > 1) std::clog << " (" << shards << " tile shards on " << opt.gpus << " device(s))";
  std::clog << "\n";

  mkdir("output", 0755);
  std::string path = "output/" + opt.output;
  FILE *f = std::fopen(path.c_str(), "wb");
  if (!f) {
    std::cerr << "[ERROR] Failed to open " << path << " for writing.\n";
    return 1;
  }
  std::string buf;
  buf.reserve((size_t)W * H * 12 + 32);
  buf += "P3\n" + std::to_string(W) + ' ' + std::to_string(H) + "\n255\n";
  const double scale = frame.pixel_samples_scale;
  char line[32];
  for (size_t px = 0; px < (size_t)W * H; ++px) {
    int n = std::snprintf(line, sizeof line, "%d %d %d\n", to_byte(scale * sum[3 * px]),
                          to_byte(scale * sum[3 * px + 1]), to_byte(scale * sum[3 * px + 2]));
    buf.append(line, (size_t)n);
  }
  std::fwrite(buf.data(), 1, buf.size(), f);
  std::fclose(f);
  std::clog << "Wrote " << path << "\n";
  return 0;
}
