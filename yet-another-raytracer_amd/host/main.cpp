// main.cpp — `yart` CLI: the reference's `raytracer --scene ...` (main.rs:777-781) on MI355X.
// Same flags and per-scene defaults (main.rs:78-107, 211-432); the render loop runs through the
// C ABI of libyart.so. Extensions: --seed (RNG key), --gpus N (pixel blocks dealt round-robin
// over N devices from one process and gathered to device 0 with one RCCL gather,
// yart_render_multi), --assets DIR (reference input meshes).
// --workers is accepted for compatibility and has no effect on the GPU path.
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <unistd.h>
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

// The reference's indicatif bar (main.rs:735-761): "Rendering [elapsed] [bar] pct pos/len px",
// fed from yart_render's progress callback (on this thread); drawn only on a terminal.
struct Bar {
  uint64_t total;
  bool tty = isatty(2) != 0;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  static void cb(uint64_t px, void* user) { static_cast<Bar*>(user)->draw(px); }
  void draw(uint64_t px) {
    if (!tty || total == 0) return;
    const int w = 28, fill = (int)(w * px / total);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "\r   Rendering [%7.1fs] [", s);
    for (int i = 0; i < w; ++i) std::fputc(i < fill ? '=' : (i == fill ? '>' : ' '), stderr);
    std::fprintf(stderr, "] %3d%% %7llu/%-7llu px", (int)(100 * px / total), (unsigned long long)px,
                 (unsigned long long)total);
    std::fflush(stderr);
  }
  void finish() {  // finish_and_clear
    if (tty) std::fprintf(stderr, "\r%*s\r", 90, "");
  }
};

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
  if (gpus > ndev) {
    std::fprintf(stderr, "warning: --gpus %d but only %d device%s visible; using %d\n", gpus, ndev, ndev > 1 ? "s" : "",
                 ndev);
    gpus = ndev;
  }
  const size_t n3 = 3 * (size_t)o.width * o.height;
  std::vector<double> xyz(n3, 0.0);
  yart_render_params p{o.width, o.height, (uint32_t)o.samples_per_pixel, (uint32_t)o.max_depth, 0x59415254ull, 0, 1, 0, 0};
  if (cli.seed) p.seed = cli.seed;
  Bar bar{(uint64_t)o.width * o.height};
  int rc;
  if (cli.gpus > 0) {
    // --gpus N: one scene per device, shards rendered at once, ONE RCCL gather to device 0
    std::vector<int> devs(gpus);
    for (int g = 0; g < gpus; ++g) devs[g] = g;
    yart_multi* m = nullptr;
    rc = yart_multi_create(gpus, devs.data(), yart_preset_desc(preset), &m);
    if (rc == YART_OK) rc = yart_render_multi(m, &cam, &p, xyz.data(), &Bar::cb, &bar);
    yart_multi_destroy(m);
  } else {
    yart_scene* s = nullptr;
    rc = yart_scene_create(0, yart_preset_desc(preset), &s);
    if (rc == YART_OK) rc = yart_render(s, &cam, &p, xyz.data(), &Bar::cb, &bar);
    yart_scene_destroy(s);
  }
  bar.finish();
  if (rc != YART_OK) {
    std::fprintf(stderr, "error: %s\n", yart_last_error());
    return 1;
  }
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
