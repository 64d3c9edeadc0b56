// toml_check — reads a config.toml with the reference's toml11 (configLoader.h
// parse_config) and prints every key the reference's two mains read, using the
// same accessors (photon-mapping/src/hostCode.cu:153-158,
// ray-tracer/src/hostCode.cu:193-206; toml_to_vec3f / toml_to_vec2i of
// configLoader.h:22-30). One line per key: "<table.key> <value...>" or
// "<table.key> ERR". A parse failure prints "PARSE_ERROR".
#include <cstdio>
#include <string>

#include "toml.hpp"

static void vec3(const toml::value& c, const char* t, const char* k) {
  try {
    const auto& a = c.at(t).at(k).as_array();
    std::printf("%s.%s %.9g %.9g %.9g\n", t, k, (float)a.at(0).as_floating(), (float)a.at(1).as_floating(),
                (float)a.at(2).as_floating());
  } catch (const std::exception&) {
    std::printf("%s.%s ERR\n", t, k);
  }
}
static void vec2i(const toml::value& c, const char* t, const char* k) {
  try {
    const auto& a = c.at(t).at(k).as_array();
    std::printf("%s.%s %d %d\n", t, k, (int)a.at(0).as_integer(), (int)a.at(1).as_integer());
  } catch (const std::exception&) {
    std::printf("%s.%s ERR\n", t, k);
  }
}
static void str(const toml::value& c, const char* t, const char* k) {
  try {
    std::printf("%s.%s %s\n", t, k, c.at(t).at(k).as_string().c_str());
  } catch (const std::exception&) {
    std::printf("%s.%s ERR\n", t, k);
  }
}
static void integer(const toml::value& c, const char* t, const char* k) {
  try {
    std::printf("%s.%s %lld\n", t, k, (long long)c.at(t).at(k).as_integer());
  } catch (const std::exception&) {
    std::printf("%s.%s ERR\n", t, k);
  }
}
static void floating(const toml::value& c, const char* t, const char* k) {
  try {
    std::printf("%s.%s %.9g\n", t, k, (float)c.at(t).at(k).as_floating());
  } catch (const std::exception&) {
    std::printf("%s.%s ERR\n", t, k);
  }
}

int main(int argc, char** argv) {
  if (argc != 2) return 2;
  toml::value c;
  try {
    c = toml::parse(argv[1]);
  } catch (const std::exception&) {
    std::printf("PARSE_ERROR\n");
    return 0;
  }
  vec3(c, "camera", "look_from");
  vec3(c, "camera", "look_at");
  vec3(c, "camera", "look_up");
  floating(c, "camera", "fovy");
  str(c, "data", "photons_file");
  str(c, "data", "caustics_photons_file");
  str(c, "data", "model_path");
  vec3(c, "ray-tracer", "sky_colour");
  str(c, "ray-tracer", "output_filename");
  vec2i(c, "ray-tracer", "fb_size");
  integer(c, "ray-tracer", "samples_per_pixel");
  integer(c, "ray-tracer", "depth");
  integer(c, "photon-mapper", "max_depth");
  integer(c, "photon-mapper", "casted_diffuse_photons");
  integer(c, "photon-mapper", "casted_caustics_photons");
  return 0;
}
