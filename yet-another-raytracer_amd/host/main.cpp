// main.cpp — `yart` CLI: the reference's `raytracer --scene ...` (main.rs:777-781) on MI355X.
// Same flags and per-scene defaults (main.rs:78-107, 211-432); the render loop runs through the
// C ABI of libyart.so. Extensions: --seed (RNG key), --gpus N (pixel blocks dealt round-robin
// over N devices from one process, summed on the host), --assets DIR (reference input meshes).
// --workers is accepted for compatibility and has no effect on the GPU path.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "../../include/yart.h"
#include "../../include/yart_host.h"

static std::string dirname_of(const std::string& p) {
  size_t s = p.find_last_of('/');
  return s == std::string::npos ? std::string() : p.substr(0, s);
}
static void mkdirs(const std::string& d) {
  if (d.empty()) return;
  std::string cur;
  for (size_t i = 0; i <= d.size(); ++i) {
    if (i == d.size() || d[i] == '/') {
      if (!cur.empty()) ::mkdir(cur.c_str(), 0755);
    }
    if (i < d.size()) cur += d[i];
  }
}

static const char kUsage[] =
    "Usage: yart --scene <SCENE> [--output <OUTPUT>] [--width <WIDTH>] [--height <HEIGHT>] "
    "[--samples <SAMPLES>] [--max-depth <MAX_DEPTH>] [--workers <WORKERS>] [--vfov <VFOV>] "
    "[--aperture <APERTURE>] [--seed <SEED>] [--gpus <GPUS>] [--assets <DIR>]\n";

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {  // clap's -h / --help (main.rs:78-107 derives Parser)
    if (std::strcmp(argv[i], "-h") == 0 || std::strcmp(argv[i], "--help") == 0) {
      std::fputs(kUsage, stdout);
      return 0;
    }
  }
  yart_cli cli;
  if (yart_cli_parse(argc, (const char* const*)argv, &cli) != YART_OK) {
    std::fprintf(stderr, "error: %s\n\n%s", yart_host_last_error(), kUsage);
    return 2;
  }
  std::string assets = cli.assets[0] ? cli.assets : "assets";
  yart_preset* preset = nullptr;
  if (yart_preset_create(cli.scene, assets.c_str(), 42, &preset) != YART_OK) {
    std::fprintf(stderr, "error: %s\n", yart_host_last_error());
    return 1;
  }
  if (yart_preset_stand_in(preset)[0]) std::fprintf(stderr, "note: %s\n", yart_preset_stand_in(preset));
  yart_render_defaults d;
  yart_preset_defaults(preset, &d);
  yart_render_options o;
  yart_resolve_render_options(d.output_filename, &d, &cli, &o);

  auto t0 = std::chrono::steady_clock::now();
  yart_camera cam;  // render() (main.rs:610-626)
  const double vup[3] = {0.0, 1.0, 0.0};
  yart_camera_init(&cam, d.lookfrom, d.lookat, vup, o.vfov, (double)o.width / (double)o.height, o.aperture, 10.0, 0.0, 1.0);

  int ndev = 0;
  if (yart_device_count(&ndev) != YART_OK || ndev == 0) {
    std::fprintf(stderr, "error: no HIP device: %s\n", yart_last_error());
    return 1;
  }
  int gpus = cli.gpus > 0 ? cli.gpus : 1;
  if (gpus > ndev) gpus = ndev;
  const size_t n3 = 3 * (size_t)o.width * o.height;
  std::vector<std::vector<double>> parts(gpus, std::vector<double>(n3, 0.0));
  std::vector<int> rcs(gpus, 0);
  std::vector<std::string> errs(gpus);
  std::vector<std::thread> th;
  for (int g = 0; g < gpus; ++g)
    th.emplace_back([&, g] {
      yart_scene* s = nullptr;
      rcs[g] = yart_scene_create(g, yart_preset_desc(preset), &s);
      if (rcs[g] == YART_OK) {
        yart_render_params p{o.width, o.height, (uint32_t)o.samples_per_pixel, (uint32_t)o.max_depth, 0x59415254ull,
                             (uint32_t)g, (uint32_t)gpus, 0, 0};
        if (cli.seed) p.seed = cli.seed;
        rcs[g] = yart_render(s, &cam, &p, parts[g].data(), nullptr, nullptr);
      }
      if (rcs[g] != YART_OK) errs[g] = yart_last_error();
      yart_scene_destroy(s);
    });
  for (auto& t : th) t.join();
  for (int g = 0; g < gpus; ++g)
    if (rcs[g] != YART_OK) {
      std::fprintf(stderr, "error: device %d: %s\n", g, errs[g].c_str());
      return 1;
    }
  std::vector<double> xyz(n3, 0.0);
  for (int g = 0; g < gpus; ++g)
    for (size_t i = 0; i < n3; ++i) xyz[i] = xyz[i] + parts[g][i];  // one writer per pixel: exact
  std::vector<uint8_t> rgba(4 * (size_t)o.width * o.height);
  if (yart_finalize_rgba8(0, xyz.data(), o.width, o.height, (uint32_t)o.samples_per_pixel, rgba.data()) != YART_OK) {
    std::fprintf(stderr, "error: %s\n", yart_last_error());
    return 1;
  }
  double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("%s rendered in %d seconds (%.3f s, %.1f Msamples/s on %d GPU%s)\n", o.output_path, (int)secs, secs,
              (double)o.width * o.height * o.samples_per_pixel / secs / 1e6, gpus, gpus > 1 ? "s" : "");
  mkdirs(dirname_of(o.output_path));
  if (yart_write_png(o.output_path, rgba.data(), o.width, o.height) != YART_OK) {
    std::fprintf(stderr, "error: could not write %s\n", o.output_path);
    return 1;
  }
  yart_preset_destroy(preset);
  return 0;
}
