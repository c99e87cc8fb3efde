// gen_scenes.cpp — writes the JSON scene files of the benchmark configurations.
//
// The reference hard-codes its scenes (src/main.cpp:21-131) and draws the
// bouncing-spheres layout and the Perlin tables from its global mt19937
// (Utility.hpp:16-37, PerlinNoise.hpp:19-26).  This tool regenerates them with the
// same libstdc++ engine and distributions, seeded, in g++'s evaluation order
// (constructor / operator arguments right to left), and prints %.17g numbers so
// the JSON round-trips exactly.
//
//   gen_scenes <three_spheres|cornell|bouncing|cornell_fog> [seed]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

static std::mt19937 eng;
static double rd() { return std::uniform_real_distribution<double>(0.0, 1.0)(eng); }
static double rd(double a, double b) { return std::uniform_real_distribution<double>(a, b)(eng); }
static int ri(int a, int b) { return std::uniform_int_distribution<int>(a, b)(eng); }

struct V {
  double x, y, z;
};
static std::string g(double v) {
  char b[64];
  snprintf(b, sizeof b, "%.17g", v);
  return b;
}
static std::string j(V v) { return "[" + g(v.x) + ", " + g(v.y) + ", " + g(v.z) + "]"; }
static V rand_vec(double a, double b) { // Vec3::random(min,max): z, y, x
  double z = rd(a, b), y = rd(a, b), x = rd(a, b);
  return V{x, y, z};
}

static std::string perlin_json() { // PerlinNoise() constructor draw order
  std::string s = "{\"rand_vec\": [";
  for (int i = 0; i < 256; ++i) {
    V v = rand_vec(-1, 1);
    double l = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    V u = (l > 1e-8) ? V{v.x * (1.0 / l), v.y * (1.0 / l), v.z * (1.0 / l)} : V{1, 0, 0};
    s += (i ? ", " : "") + j(u);
  }
  s += "]";
  const char *names[3] = {"perm_x", "perm_y", "perm_z"};
  for (int a = 0; a < 3; ++a) {
    int p[256];
    for (int i = 0; i < 256; ++i) p[i] = i;
    for (int i = 255; i > 0; i--) {
      int t = ri(0, i);
      int tmp = p[i];
      p[i] = p[t];
      p[t] = tmp;
    }
    s += std::string(", \"") + names[a] + "\": [";
    for (int i = 0; i < 256; ++i) s += (i ? ", " : "") + std::to_string(p[i]);
    s += "]";
  }
  return s + "}";
}

static void three_spheres() {
  // BASELINE.json config 1: "default JSON scene (3 spheres, Lambertian)" 
  printf("{\n  \"name\": \"three_spheres\",\n");
  printf("  \"camera\": {\"image_width\": 400, \"aspect_ratio\": %s, \"samples_per_pixel\": 10,"
         " \"max_depth\": 8, \"vfov\": 90, \"lookfrom\": [0, 0, 0], \"lookat\": [0, 0, -1],"
         " \"vup\": [0, 1, 0], \"defocus_angle\": 0, \"focus_dist\": 10,"
         " \"background\": [0.7, 0.8, 1.0]},\n",
         g(16.0 / 9.0).c_str());
  printf("  \"use_bvh\": false,\n");
  printf("  \"materials\": {\n"
         "    \"ground\": {\"type\": \"lambertian\", \"albedo\": [0.8, 0.8, 0.0]},\n"
         "    \"center\": {\"type\": \"lambertian\", \"albedo\": [0.1, 0.2, 0.5]},\n"
         "    \"left\": {\"type\": \"lambertian\", \"albedo\": [0.8, 0.3, 0.3]}\n  },\n");
  printf("  \"world\": [\n"
         "    {\"type\": \"sphere\", \"center\": [0, -100.5, -1], \"radius\": 100, \"material\": \"ground\"},\n"
         "    {\"type\": \"sphere\", \"center\": [0, 0, -1.2], \"radius\": 0.5, \"material\": \"center\"},\n"
         "    {\"type\": \"sphere\", \"center\": [-1, 0, -1], \"radius\": 0.5, \"material\": \"left\"}\n"
         "  ],\n  \"lights\": []\n}\n");
}

static void cornell_body(bool fog, unsigned seed) {
  // populate_cornell_box_scene, main.cpp:21-71
  printf("  \"materials\": {\n"
         "    \"red\": {\"type\": \"lambertian\", \"albedo\": [0.65, 0.05, 0.05]},\n"
         "    \"white\": {\"type\": \"lambertian\", \"albedo\": [0.73, 0.73, 0.73]},\n"
         "    \"green\": {\"type\": \"lambertian\", \"albedo\": [0.12, 0.45, 0.15]},\n"
         "    \"light\": {\"type\": \"diffuse_light\", \"emit\": [15, 15, 15]},\n"
         "    \"glass\": {\"type\": \"dielectric\", \"refraction_index\": 1.5}\n  },\n");
  if (fog) {
    eng.seed(seed);
    printf("  \"perlin\": {\"fog\": %s},\n", perlin_json().c_str());
    printf("  \"textures\": {\"fog\": {\"type\": \"noise\", \"scale\": 0.1, \"perlin\": \"fog\"}},\n");
  }
  printf("  \"world\": [\n"
         "    {\"type\": \"quad\", \"Q\": [555, 0, 0], \"u\": [0, 0, 555], \"v\": [0, 555, 0], \"material\": \"green\"},\n"
         "    {\"type\": \"quad\", \"Q\": [0, 0, 555], \"u\": [0, 0, -555], \"v\": [0, 555, 0], \"material\": \"red\"},\n"
         "    {\"type\": \"quad\", \"Q\": [0, 555, 0], \"u\": [555, 0, 0], \"v\": [0, 0, 555], \"material\": \"white\"},\n"
         "    {\"type\": \"quad\", \"Q\": [0, 0, 555], \"u\": [555, 0, 0], \"v\": [0, 0, -555], \"material\": \"white\"},\n"
         "    {\"type\": \"quad\", \"Q\": [555, 0, 555], \"u\": [-555, 0, 0], \"v\": [0, 555, 0], \"material\": \"white\"},\n"
         "    {\"type\": \"quad\", \"Q\": [213, 554, 227], \"u\": [130, 0, 0], \"v\": [0, 0, 105], \"material\": \"light\"},\n");
  const char *box = "{\"type\": \"translate\", \"offset\": [265, 0, 295], \"object\": "
                    "{\"type\": \"rotate_y\", \"angle\": 15, \"object\": "
                    "{\"type\": \"box\", \"a\": [0, 0, 0], \"b\": [165, 330, 165], \"material\": \"white\"}}}";
  if (fog)
    printf("    {\"type\": \"constant_medium\", \"density\": 0.01, \"texture\": \"fog\", \"boundary\": %s},\n", box);
  else
    printf("    %s,\n", box);
  printf("    {\"type\": \"sphere\", \"center\": [190, 90, 190], \"radius\": 90, \"material\": \"glass\"}\n  ],\n");
  printf("  \"lights\": [\n"
         "    {\"type\": \"quad\", \"Q\": [343, 554, 332], \"u\": [-130, 0, 0], \"v\": [0, 0, -105]},\n"
         "    {\"type\": \"sphere\", \"center\": [190, 90, 190], \"radius\": 90}\n  ]\n}\n");
}

static void cornell() {
  printf("{\n  \"name\": \"cornell\",\n");
  printf("  \"camera\": {\"image_width\": 600, \"aspect_ratio\": 1.0, \"samples_per_pixel\": 100,"
         " \"max_depth\": 50, \"vfov\": 40, \"lookfrom\": [278, 278, -800], \"lookat\": [278, 278, 0],"
         " \"vup\": [0, 1, 0], \"defocus_angle\": 0, \"focus_dist\": 10, \"background\": [0, 0, 0]},\n");
  printf("  \"use_bvh\": false,\n");
  cornell_body(false, 0);
}

static void cornell_fog(unsigned seed) {
  // BASELINE.json config 4: Cornell + emissive + dielectric + Perlin fog, 16:9
  printf("{\n  \"name\": \"cornell_fog\",\n");
  printf("  \"camera\": {\"image_width\": 1920, \"aspect_ratio\": %s, \"samples_per_pixel\": 1024,"
         " \"max_depth\": 8, \"vfov\": 40, \"lookfrom\": [278, 278, -800], \"lookat\": [278, 278, 0],"
         " \"vup\": [0, 1, 0], \"defocus_angle\": 0, \"focus_dist\": 10, \"background\": [0, 0, 0]},\n",
         g(16.0 / 9.0).c_str());
  printf("  \"use_bvh\": true,\n");
  cornell_body(true, seed);
}

static void bouncing(unsigned seed) {
  // populate_bouncing_spheres_scene, main.cpp:73-131
  eng.seed(seed);
  std::vector<std::string> objs, mats;
  objs.push_back("{\"type\": \"sphere\", \"center\": [0, -1000, 0], \"radius\": 1000, \"material\": \"ground\"}");
  int n = 0;
  for (int a = -11; a < 11; a++)
    for (int b = -11; b < 11; b++) {
      double choose = rd();
      double cz = b + 0.9 * rd(); // Point3(x, y, z): z argument evaluated first
      double cx = a + 0.9 * rd();
      V c{cx, 0.2, cz};
      double dx = c.x - 4, dy = c.y - 0.2, dz = c.z - 0;
      if (std::sqrt(dx * dx + dy * dy + dz * dz) > 0.9) {
        std::string m = "m" + std::to_string(n++);
        if (choose < 0.8) {
          V r2 = rand_vec(0, 1); // Color::random() * Color::random(): right operand first
          V r1 = rand_vec(0, 1);
          V alb{r1.x * r2.x, r1.y * r2.y, r1.z * r2.z};
          mats.push_back("\"" + m + "\": {\"type\": \"lambertian\", \"albedo\": " + j(alb) + "}");
          double up = rd(0, .5);
          V c2{c.x + 0, c.y + up, c.z + 0};
          objs.push_back("{\"type\": \"sphere\", \"center\": " + j(c) + ", \"center2\": " + j(c2) +
                         ", \"radius\": 0.2, \"material\": \"" + m + "\"}");
        } else if (choose < 0.95) {
          V alb = rand_vec(0.5, 1);
          double fuzz = rd(0, 0.5);
          mats.push_back("\"" + m + "\": {\"type\": \"metal\", \"albedo\": " + j(alb) +
                         ", \"fuzz\": " + g(fuzz) + "}");
          objs.push_back("{\"type\": \"sphere\", \"center\": " + j(c) + ", \"radius\": 0.2, \"material\": \"" + m + "\"}");
        } else {
          mats.push_back("\"" + m + "\": {\"type\": \"dielectric\", \"refraction_index\": 1.5}");
          objs.push_back("{\"type\": \"sphere\", \"center\": " + j(c) + ", \"radius\": 0.2, \"material\": \"" + m + "\"}");
        }
      }
    }
  mats.push_back("\"glass\": {\"type\": \"dielectric\", \"refraction_index\": 1.5}");
  mats.push_back("\"brown\": {\"type\": \"lambertian\", \"albedo\": [0.4, 0.2, 0.1]}");
  mats.push_back("\"mirror\": {\"type\": \"metal\", \"albedo\": [0.7, 0.6, 0.5], \"fuzz\": 0.0}");
  mats.push_back("\"ground\": {\"type\": \"lambertian\", \"texture\": \"checker\"}");
  objs.push_back("{\"type\": \"sphere\", \"center\": [0, 1, 0], \"radius\": 1.0, \"material\": \"glass\"}");
  objs.push_back("{\"type\": \"sphere\", \"center\": [-4, 1, 0], \"radius\": 1.0, \"material\": \"brown\"}");
  objs.push_back("{\"type\": \"sphere\", \"center\": [4, 1, 0], \"radius\": 1.0, \"material\": \"mirror\"}");
  printf("{\n  \"name\": \"bouncing_seed%u\",\n", seed);
  printf("  \"camera\": {\"image_width\": 1920, \"aspect_ratio\": %s, \"samples_per_pixel\": 256,"
         " \"max_depth\": 8, \"vfov\": 20, \"lookfrom\": [13, 2, 3], \"lookat\": [0, 0, 0],"
         " \"vup\": [0, 1, 0], \"defocus_angle\": 0.6, \"focus_dist\": 10.0,"
         " \"background\": [0.7, 0.8, 1.0]},\n",
         g(16.0 / 9.0).c_str());
  printf("  \"use_bvh\": true,\n");
  printf("  \"textures\": {\"checker\": {\"type\": \"checker\", \"scale\": 0.32, \"even\": \"ce\", \"odd\": \"co\"},"
         " \"ce\": {\"type\": \"solid\", \"color\": [0.2, 0.3, 0.1]},"
         " \"co\": {\"type\": \"solid\", \"color\": [0.9, 0.9, 0.9]}},\n");
  printf("  \"materials\": {\n");
  for (size_t i = 0; i < mats.size(); ++i) printf("    %s%s\n", mats[i].c_str(), i + 1 < mats.size() ? "," : "");
  printf("  },\n  \"world\": [\n");
  for (size_t i = 0; i < objs.size(); ++i) printf("    %s%s\n", objs[i].c_str(), i + 1 < objs.size() ? "," : "");
  printf("  ],\n  \"lights\": []\n}\n");
  fprintf(stderr, "bouncing seed %u: %zu objects\n", seed, objs.size());
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: gen_scenes <three_spheres|cornell|bouncing|cornell_fog> [seed]\n");
    return 2;
  }
  unsigned seed = argc > 2 ? (unsigned)strtoul(argv[2], nullptr, 10) : 42u;
  std::string w = argv[1];
  if (w == "three_spheres") three_spheres();
  else if (w == "cornell") cornell();
  else if (w == "bouncing") bouncing(seed);
  else if (w == "cornell_fog") cornell_fog(seed);
  else return 2;
  return 0;
}
