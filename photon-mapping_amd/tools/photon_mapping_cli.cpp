// photon_mapping_cli.cpp — the B1 process contract on top of
// the C-ABI in include/pm.h. One binary, three names:
//
//   photonMapping   stage 1 (photon-mapping/src/hostCode.cu:140-186): trace
//                   the diffuse and caustic photon maps and write them as %.6f
//                   text to data.photons_file / data.caustics_photons_file.
//   rayTracer       stage 2 (ray-tracer/src/hostCode.cu:180-245): read both
//                   photon files, build the kd-trees, render, write
//                   ray-tracer.output_filename (RGBA8 PNG, row H-y layout).
//   photonViewer    photon-viewer/src/hostCode.cu:156-177: splat both photon
//                   files onto photon-viewer.fb_size images (visibility rays),
//                   written to photon-viewer.output_filename /
//                   caustics_output_filename.
//   photon-mapping  both stages in one process. The photon files are written
//                   and their %.6f round trip is applied on the device
//                   (pm_photons_quantize), so the image equals the two-process
//                   reference pipeline; --in-memory renders the unquantised
//                   photons.
//
// The config is ../config.toml relative to the working directory
// (configLoader.h:6), overridable with --config PATH. All compute runs on the
// GPU through libpm_hip.so; there is no CPU path.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pm.h"

namespace {

using Clock = std::chrono::steady_clock;

double ms_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

[[noreturn]] void die(const char* what, int st) {
  std::fprintf(stderr, "photon-mapping: %s failed: %s\n", what, pm_status_string(st));
  std::exit(1);
}

void check(int st, const char* what) {
  if (st != PM_OK) die(what, st);
}

// Device buffer owned through the C-ABI allocation helpers.
struct DevMem {
  void* p = nullptr;
  DevMem() = default;
  explicit DevMem(size_t bytes) { check(pm_device_alloc(bytes, &p), "device allocation"); }
  ~DevMem() { pm_device_free(p); }
  DevMem(const DevMem&) = delete;
  DevMem& operator=(const DevMem&) = delete;
};

struct Scene {
  pm_scene_data* data = nullptr;
  const pm_mesh* meshes = nullptr;
  const pm_light* lights = nullptr;
  int32_t nmesh = 0, nlight = 0;
  pm_scene* gpu = nullptr;
  ~Scene() {
    if (gpu) pm_scene_destroy(gpu);
    if (data) pm_scene_data_free(data);
  }
};

void load_scene(const pm_config& cfg, Scene& sc) {
  check(pm_scene_data_load(cfg.model_path, &sc.data), "import_scene");
  int64_t nv = 0, nt = 0;
  pm_scene_data_counts(sc.data, &sc.nmesh, &sc.nlight, &nv, &nt);
  pm_scene_data_meshes(sc.data, &sc.meshes);
  pm_scene_data_lights(sc.data, &sc.lights);
  std::printf("Loaded world: %d meshes, %lld triangles, %d lights.\n", sc.nmesh, (long long)nt, sc.nlight);
  const auto t0 = Clock::now();
  check(pm_scene_create(sc.meshes, sc.nmesh, &sc.gpu), "loadGeometry (LBVH build)");
  std::printf("Built BVH in %.1f ms.\n", ms_since(t0));
}

// runNormal / runCaustics (photon-mapping/src/hostCode.cu:112-138): returns the
// photons on the host.
std::vector<pm_photon> trace(const Scene& sc, const pm_config& cfg, bool caustics) {
  pm_trace_params p{};
  p.casted_photons = caustics ? cfg.casted_caustics_photons : cfg.casted_diffuse_photons;
  p.max_depth = cfg.max_depth;
  p.caustics_mode = caustics ? 1 : 0;
  p.shard_rank = 0;
  p.shard_count = 1;
  int64_t cap = 0, count = 0;
  check(pm_trace_capacity(sc.lights, sc.nlight, &p, &cap), "trace capacity");
  DevMem d(sizeof(pm_photon) * (size_t)(cap > 0 ? cap : 1));
  const auto t0 = Clock::now();
  check(pm_trace_photons(sc.gpu, sc.lights, sc.nlight, &p, static_cast<pm_photon*>(d.p), cap, &count, nullptr),
        caustics ? "runCaustics" : "runNormal");
  std::printf("%s: %lld photons stored in %.1f ms.\n", caustics ? "Caustics" : "Global", (long long)count,
              ms_since(t0));
  std::vector<pm_photon> h((size_t)count);
  check(pm_copy_to_host(h.data(), d.p, sizeof(pm_photon) * (size_t)count), "photon copy");
  return h;
}

// readPhotonsFromFile (ray-tracer/src/hostCode.cu:26-52): a missing file is
// reported on stderr and yields no photons.
std::vector<pm_photon> read_photons(const char* path) {
  pm_photon* h = nullptr;
  int64_t n = 0;
  const int st = pm_photons_read_txt(path, &h, &n);
  if (st == PM_ERR_IO) {
    std::fprintf(stderr, "Error opening file: %s\n", path);
    return {};
  }
  check(st, "readPhotonsFromFile");
  std::vector<pm_photon> v(h, h + n);
  pm_free(h);
  return v;
}

// photonViewer run() (photon-viewer/src/hostCode.cu:109-154) for one photon file
int view_file(const pm_config& cfg, const Scene& sc, const char* photons_path, const char* out_path) {
  const std::vector<pm_photon> ph = read_photons(photons_path);
  const int W = cfg.viewer_fb_width, H = cfg.viewer_fb_height;
  DevMem dp(sizeof(pm_photon) * (ph.size() ? ph.size() : 1)), fb(sizeof(uint32_t) * (size_t)W * (size_t)H);
  check(pm_copy_to_device(dp.p, ph.data(), sizeof(pm_photon) * ph.size()), "photon upload");
  pm_viewer_params vp{cfg.look_from, cfg.look_at, cfg.look_up, cfg.fovy, W, H};
  check(pm_photon_view(sc.gpu, static_cast<pm_photon*>(dp.p), (int64_t)ph.size(), &vp, static_cast<uint32_t*>(fb.p),
                       nullptr),
        "photonViewerRayGen");
  std::vector<uint32_t> h((size_t)W * (size_t)H);
  check(pm_copy_to_host(h.data(), fb.p, sizeof(uint32_t) * h.size()), "framebuffer copy");
  check(pm_write_png_rgba(out_path, h.data(), W, H), "stbi_write_png");
  std::printf("Saved %s (%zu photons, %dx%d).\n", out_path, ph.size(), W, H);
  return 0;
}

int stage_photons(const pm_config& cfg, const Scene& sc, std::vector<pm_photon>* g_out,
                  std::vector<pm_photon>* c_out) {
  std::vector<pm_photon> g = trace(sc, cfg, false);
  check(pm_photons_write_txt(cfg.photons_file, g.data(), (int64_t)g.size()), "writeAlivePhotons (global)");
  std::vector<pm_photon> c = trace(sc, cfg, true);
  check(pm_photons_write_txt(cfg.caustics_photons_file, c.data(), (int64_t)c.size()), "writeAlivePhotons (caustics)");
  if (g_out) *g_out = std::move(g);
  if (c_out) *c_out = std::move(c);
  return 0;
}

int stage_render(const pm_config& cfg, const Scene& sc, const std::vector<pm_photon>& g,
                 const std::vector<pm_photon>& c, bool quantize) {
  std::printf("Loaded %lld photons (non-caustic %lld, caustic %lld).\n", (long long)(g.size() + c.size()),
              (long long)g.size(), (long long)c.size());
  DevMem dg(sizeof(pm_photon) * (g.size() ? g.size() : 1)), dc(sizeof(pm_photon) * (c.size() ? c.size() : 1));
  check(pm_copy_to_device(dg.p, g.data(), sizeof(pm_photon) * g.size()), "photon upload");
  check(pm_copy_to_device(dc.p, c.data(), sizeof(pm_photon) * c.size()), "photon upload");
  if (quantize) {   // the %.6f file round trip, applied on the device
    check(pm_photons_quantize(static_cast<pm_photon*>(dg.p), (int64_t)g.size(), nullptr), "quantize");
    check(pm_photons_quantize(static_cast<pm_photon*>(dc.p), (int64_t)c.size(), nullptr), "quantize");
  }
  // loadPhotons (ray-tracer/src/hostCode.cu:54-99): global = diffuse (power 1)
  // ++ caustic (power 0.5); caustic map = caustic (power 0.5).
  pm_photon_map *gm = nullptr, *cm = nullptr;
  auto t0 = Clock::now();
  check(pm_photon_map_create(static_cast<pm_photon*>(dg.p), (int64_t)g.size(), 1.0f, static_cast<pm_photon*>(dc.p),
                             (int64_t)c.size(), 0.5f, &gm, nullptr),
        "buildTree (global)");
  check(pm_photon_map_create(static_cast<pm_photon*>(dc.p), (int64_t)c.size(), 0.5f, nullptr, 0, 0.0f, &cm, nullptr),
        "buildTree (caustic)");
  std::printf("Time taken to build KD-Tree: %.1f ms\n", ms_since(t0));

  const int W = cfg.fb_width, H = cfg.fb_height;
  pm_render_params rp{};
  rp.width = W;
  rp.height = H;
  rp.samples_per_pixel = cfg.samples_per_pixel;
  rp.max_depth = cfg.depth;
  check(pm_camera_setup(cfg.look_from, cfg.look_at, cfg.look_up, cfg.fovy, W, H, &rp.camera), "setupCamera");
  rp.sky_colour = cfg.sky_colour;
  rp.tile_rank = 0;
  rp.tile_count = 1;
  DevMem fb(sizeof(uint32_t) * (size_t)W * (size_t)H);
  std::vector<uint32_t> zero((size_t)W * (size_t)H, 0u);   // row 0 is never written (deviceCode.cu:224-229)
  check(pm_copy_to_device(fb.p, zero.data(), sizeof(uint32_t) * zero.size()), "framebuffer clear");
  t0 = Clock::now();
  check(pm_render(sc.gpu, &rp, sc.lights, sc.nlight, gm, cm, static_cast<uint32_t*>(fb.p), nullptr, nullptr),
        "render");
  std::printf("Time taken to render: %.1f ms\n", ms_since(t0));
  std::vector<uint32_t> h((size_t)W * (size_t)H);
  check(pm_copy_to_host(h.data(), fb.p, sizeof(uint32_t) * h.size()), "framebuffer copy");
  check(pm_write_png_rgba(cfg.output_filename, h.data(), W, H), "stbi_write_png");
  pm_photon_map_destroy(gm);
  pm_photon_map_destroy(cm);
  std::printf("Saved %s (%dx%d).\n", cfg.output_filename, W, H);
  return 0;
}

// toml11's as_* on an absent key throws and ends the reference process; here
// the stage's keys are checked up front instead.
bool require_keys(const pm_config& cfg, const std::vector<const char*>& keys) {
  bool ok = true;
  for (const char* k : keys) {
    int idx = -1;
    for (int i = 0; pm_config_key_name(i); i++)
      if (std::strcmp(pm_config_key_name(i), k) == 0) idx = i;
    if (idx < 0 || !(cfg.present_mask & (1u << idx))) {
      std::fprintf(stderr, "config: missing key %s\n", k);
      ok = false;
    }
  }
  return ok;
}

void usage(const char* prog) {
  std::fprintf(stderr,
               "usage: %s [--config PATH] [--stage photons|render|all|view] [--in-memory]\n"
               "  photonMapping = --stage photons, rayTracer = --stage render, photonViewer = --stage view,\n"
               "  photon-mapping = --stage all\n",
               prog);
}

}  // namespace

int main(int argc, char** argv) {
  std::string name = argv[0];
  const size_t slash = name.find_last_of('/');
  if (slash != std::string::npos) name = name.substr(slash + 1);
  std::string stage = name == "photonMapping" ? "photons"
                      : name == "rayTracer"   ? "render"
                      : name == "photonViewer" ? "view"
                                               : "all";
  std::string config = "../config.toml";   // configLoader.h:6
  if (const char* e = std::getenv("PM_CONFIG")) config = e;
  bool in_memory = false;
  for (int i = 1; i < argc; i++) {
    const std::string a = argv[i];
    if (a == "--config" && i + 1 < argc) {
      config = argv[++i];
    } else if (a == "--stage" && i + 1 < argc) {
      stage = argv[++i];
    } else if (a == "--in-memory") {
      in_memory = true;
    } else {
      usage(argv[0]);
      return 2;
    }
  }
  if (stage != "photons" && stage != "render" && stage != "all" && stage != "view") {
    usage(argv[0]);
    return 2;
  }
  pm_config cfg{};
  const int st = pm_config_load(config.c_str(), &cfg);
  if (st != PM_OK) {
    std::fprintf(stderr, "Parsing failed:\n%s\n", cfg.error[0] ? cfg.error : pm_status_string(st));
    return 1;
  }
  std::printf("Loaded config: %s\n", config.c_str());
  std::vector<const char*> keys = {"data.photons_file", "data.caustics_photons_file", "data.model_path"};
  if (stage != "render")   // photon-mapping/src/hostCode.cu:153-158
    keys.insert(keys.end(), {"photon-mapper.casted_diffuse_photons", "photon-mapper.casted_caustics_photons",
                             "photon-mapper.max_depth"});
  if (stage == "view")  // photon-viewer/src/hostCode.cu:114-120,160-164
    keys = {"data.photons_file", "data.caustics_photons_file", "data.model_path", "camera.look_at",
            "camera.look_from", "camera.look_up", "camera.fovy", "photon-viewer.output_filename",
            "photon-viewer.caustics_output_filename", "photon-viewer.fb_size"};
  else if (stage != "photons")  // ray-tracer/src/hostCode.cu:193-206
    keys.insert(keys.end(), {"camera.look_at", "camera.look_from", "camera.look_up", "camera.fovy",
                             "ray-tracer.sky_colour", "ray-tracer.output_filename", "ray-tracer.fb_size",
                             "ray-tracer.samples_per_pixel", "ray-tracer.depth"});
  if (!require_keys(cfg, keys)) return 1;
  Scene sc;
  load_scene(cfg, sc);
  if (stage == "photons") return stage_photons(cfg, sc, nullptr, nullptr);
  if (stage == "view") {
    view_file(cfg, sc, cfg.photons_file, cfg.viewer_output_filename);
    return view_file(cfg, sc, cfg.caustics_photons_file, cfg.viewer_caustics_output_filename);
  }
  std::vector<pm_photon> g, c;
  if (stage == "all") {
    // the photon files are written as in the two-process pipeline; their %.6f
    // round trip is applied in memory instead of re-parsing them
    stage_photons(cfg, sc, &g, &c);
    return stage_render(cfg, sc, g, c, !in_memory);
  }
  g = read_photons(cfg.photons_file);
  c = read_photons(cfg.caustics_photons_file);
  return stage_render(cfg, sc, g, c, false);
}
