// config.cpp — config.toml reader for the drop-in boundary (B1).
//
// Replaces common/src/configLoader.h:8-19 (toml11 4.2.0 `toml::parse` of the
// fixed path "../config.toml") with a TOML-subset parser covering exactly what
// the reference reads: tables, bare/quoted/dotted keys, basic and literal
// strings (all basic escapes), integers (decimal with '_' separators,
// config.toml.example:26, and 0x/0o/0b), floats (incl. inf/nan), booleans,
// arrays. Cross-checked against the reference's own toml11 (oracle/ref,
// tests/test_toml_ref.py).
// Type rules follow toml11's accessors used by the reference: `as_integer()`
// rejects floats and `as_floating()` rejects integers (configLoader.h:21-29),
// so `fovy = 1` or `look_at = [1, 2, 3]` is an error, as it is upstream.
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../../include/pm.h"

namespace {

struct TVal {
  enum Kind { NONE, STR, INT, FLT, BOOL, ARR } kind = NONE;
  std::string s;
  long long i = 0;
  double f = 0;
  bool b = false;
  std::vector<TVal> a;
};

struct Parser {
  std::string src;
  size_t p = 0;
  int line = 1;
  std::string err;

  bool fail(const std::string& m) {
    if (err.empty()) err = "line " + std::to_string(line) + ": " + m;
    return false;
  }
  void skip_ws() {
    while (p < src.size() && (src[p] == ' ' || src[p] == '\t')) p++;
  }
  void skip_ws_nl_comments() {
    for (;;) {
      skip_ws();
      if (p < src.size() && src[p] == '#') {
        while (p < src.size() && src[p] != '\n') p++;
      } else if (p < src.size() && (src[p] == '\n' || src[p] == '\r')) {
        if (src[p] == '\n') line++;
        p++;
      } else {
        break;
      }
    }
  }
  bool parse_key_part(std::string& k) {
    skip_ws();
    k.clear();
    if (p < src.size() && (src[p] == '"' || src[p] == '\'')) {
      TVal v;
      if (!parse_string(v)) return false;
      k = v.s;
      return true;
    }
    while (p < src.size() && (std::isalnum((unsigned char)src[p]) || src[p] == '_' || src[p] == '-')) k += src[p++];
    if (k.empty()) return fail("expected key");
    return true;
  }
  // dotted keys (a.b = v, [a.b]) flatten to "a.b"
  bool parse_key(std::string& k) {
    if (!parse_key_part(k)) return false;
    for (;;) {
      skip_ws();
      if (p >= src.size() || src[p] != '.') return true;
      p++;
      std::string part;
      if (!parse_key_part(part)) return false;
      k += "." + part;
    }
  }
  static void utf8(std::string& out, unsigned long cp) {
    if (cp < 0x80) {
      out += (char)cp;
    } else if (cp < 0x800) {
      out += (char)(0xC0 | (cp >> 6));
      out += (char)(0x80 | (cp & 0x3F));
    } else if (cp < 0x10000) {
      out += (char)(0xE0 | (cp >> 12));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    } else {
      out += (char)(0xF0 | (cp >> 18));
      out += (char)(0x80 | ((cp >> 12) & 0x3F));
      out += (char)(0x80 | ((cp >> 6) & 0x3F));
      out += (char)(0x80 | (cp & 0x3F));
    }
  }
  bool parse_string(TVal& v) {
    char q = src[p++];
    v.kind = TVal::STR;
    while (p < src.size() && src[p] != q) {
      if (src[p] == '\n') return fail("unterminated string");
      if (q == '"' && src[p] == '\\' && p + 1 < src.size()) {
        char e = src[p + 1];
        p += 2;
        switch (e) {
          case 'n': v.s += '\n'; break;
          case 't': v.s += '\t'; break;
          case 'b': v.s += '\b'; break;
          case 'f': v.s += '\f'; break;
          case 'r': v.s += '\r'; break;
          case '\\': v.s += '\\'; break;
          case '"': v.s += '"'; break;
          case 'u':
          case 'U': {
            const size_t nd = e == 'u' ? 4 : 8;
            if (p + nd > src.size()) return fail("bad unicode escape");
            const std::string hex = src.substr(p, nd);
            for (char h : hex)
              if (!std::isxdigit((unsigned char)h)) return fail("bad unicode escape");
            utf8(v.s, std::strtoul(hex.c_str(), nullptr, 16));
            p += nd;
            break;
          }
          default: return fail(std::string("bad escape \\") + e);
        }
        continue;
      }
      v.s += src[p++];
    }
    if (p >= src.size()) return fail("unterminated string");
    p++;
    return true;
  }
  bool parse_number(TVal& v) {
    size_t b = p;
    while (p < src.size() && (std::isalnum((unsigned char)src[p]) || src[p] == '_' || src[p] == '.' ||
                              src[p] == '+' || src[p] == '-'))
      p++;
    std::string t = src.substr(b, p - b), c;
    if (t == "true" || t == "false") {
      v.kind = TVal::BOOL;
      v.b = t == "true";
      return true;
    }
    // 0x / 0o / 0b integers (no sign), underscores between digits
    int radix = 10;
    if (t.size() > 2 && t[0] == '0' && (t[1] == 'x' || t[1] == 'o' || t[1] == 'b')) radix = t[1] == 'x' ? 16 : (t[1] == 'o' ? 8 : 2);
    auto is_digit = [&](char ch) { return radix == 16 ? std::isxdigit((unsigned char)ch) != 0 : std::isdigit((unsigned char)ch) != 0; };
    for (size_t i = radix == 10 ? 0 : 2; i < t.size(); i++) {
      if (t[i] == '_') {
        // TOML: underscores only between digits
        if (i == 0 || i + 1 >= t.size() || !is_digit(t[i - 1]) || !is_digit(t[i + 1]))
          return fail("bad underscore in number '" + t + "'");
        continue;
      }
      c += t[i];
    }
    if (radix != 10) {
      char* e2 = nullptr;
      if (c.empty()) return fail("bad number '" + t + "'");
      for (char ch : c)
        if (!(radix == 16 ? std::isxdigit((unsigned char)ch) : (ch >= '0' && ch < '0' + radix)))
          return fail("bad number '" + t + "'");
      v.kind = TVal::INT;
      v.i = (long long)std::strtoull(c.c_str(), &e2, radix);
      return true;
    }
    if (c.empty()) return fail("expected value");
    std::string body = (c[0] == '+' || c[0] == '-') ? c.substr(1) : c;
    if (body == "inf" || body == "nan") {
      v.kind = TVal::FLT;
      v.f = body == "inf" ? (c[0] == '-' ? -HUGE_VAL : HUGE_VAL) : NAN;
      return true;
    }
    bool is_float = c.find_first_of(".eE") != std::string::npos;
    char* end = nullptr;
    if (is_float) {
      v.kind = TVal::FLT;
      v.f = std::strtod(c.c_str(), &end);
    } else {
      v.kind = TVal::INT;
      v.i = std::strtoll(c.c_str(), &end, 10);
    }
    if (!end || *end != 0) return fail("bad number '" + t + "'");
    return true;
  }
  bool parse_value(TVal& v) {
    skip_ws();
    if (p >= src.size()) return fail("expected value");
    char ch = src[p];
    if (ch == '"' || ch == '\'') return parse_string(v);
    if (ch == '[') {
      p++;
      v.kind = TVal::ARR;
      for (;;) {
        skip_ws_nl_comments();
        if (p < src.size() && src[p] == ']') { p++; return true; }
        TVal e;
        if (!parse_value(e)) return false;
        v.a.push_back(e);
        skip_ws_nl_comments();
        if (p < src.size() && src[p] == ',') { p++; continue; }
        if (p < src.size() && src[p] == ']') { p++; return true; }
        return fail("expected ',' or ']'");
      }
    }
    return parse_number(v);
  }
  bool parse(std::map<std::string, TVal>& out) {
    std::string table;
    for (;;) {
      skip_ws_nl_comments();
      if (p >= src.size()) return true;
      if (src[p] == '[') {
        p++;
        std::string k;
        if (!parse_key(k)) return false;
        skip_ws();
        if (p >= src.size() || src[p] != ']') return fail("expected ']'");
        p++;
        table = k;
        continue;
      }
      std::string k;
      if (!parse_key(k)) return false;
      skip_ws();
      if (p >= src.size() || src[p] != '=') return fail("expected '='");
      p++;
      TVal v;
      if (!parse_value(v)) return false;
      std::string full = table.empty() ? k : table + "." + k;
      if (out.count(full)) return fail("duplicate key " + full);
      out[full] = v;
      skip_ws();
      if (p < src.size() && src[p] == '#') continue;
      if (p < src.size() && src[p] != '\n' && src[p] != '\r') return fail("trailing characters");
    }
  }
};

const char* const kKeys[] = {
    "camera.look_from", "camera.look_at", "camera.look_up", "camera.fovy",
    "data.photons_file", "data.caustics_photons_file", "data.model_path",
    "ray-tracer.sky_colour", "ray-tracer.output_filename", "ray-tracer.fb_size",
    "ray-tracer.samples_per_pixel", "ray-tracer.depth",
    "photon-viewer.output_filename", "photon-viewer.caustics_output_filename",
    "photon-viewer.fb_size",
    "photon-mapper.max_depth", "photon-mapper.casted_diffuse_photons",
    "photon-mapper.casted_caustics_photons",
};
constexpr int kNumKeys = sizeof(kKeys) / sizeof(kKeys[0]);

void set_err(pm_config* c, const std::string& m) {
  std::snprintf(c->error, sizeof(c->error), "%s", m.c_str());
}

}  // namespace

extern "C" const char* pm_config_key_name(int32_t i) {
  return (i >= 0 && i < kNumKeys) ? kKeys[i] : nullptr;
}

extern "C" int pm_config_load(const char* path, pm_config* c) {
  if (!path || !c) return PM_ERR_INVALID;
  std::memset(c, 0, sizeof(*c));
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    set_err(c, std::string("cannot open ") + path);
    return PM_ERR_IO;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  Parser P;
  P.src = ss.str();
  std::map<std::string, TVal> kv;
  if (!P.parse(kv)) {
    set_err(c, "Parsing failed: " + P.err);
    return PM_ERR_IO;
  }
  std::string err;
  auto vec3 = [&](int key, pm_float3* out) {
    auto it = kv.find(kKeys[key]);
    if (it == kv.end()) return;
    const TVal& v = it->second;
    if (v.kind != TVal::ARR || v.a.size() < 3) { err = std::string(kKeys[key]) + ": expected array of 3 floats"; return; }
    float e[3];
    for (int i = 0; i < 3; i++) {
      if (v.a[i].kind != TVal::FLT) { err = std::string(kKeys[key]) + ": array element is not a floating value"; return; }
      e[i] = (float)v.a[i].f;
    }
    *out = {e[0], e[1], e[2]};
    c->present_mask |= 1u << key;
  };
  auto vec2i = [&](int key, int32_t* x, int32_t* y) {
    auto it = kv.find(kKeys[key]);
    if (it == kv.end()) return;
    const TVal& v = it->second;
    if (v.kind != TVal::ARR || v.a.size() < 2 || v.a[0].kind != TVal::INT || v.a[1].kind != TVal::INT) {
      err = std::string(kKeys[key]) + ": expected array of 2 integers";
      return;
    }
    *x = (int32_t)v.a[0].i;
    *y = (int32_t)v.a[1].i;
    c->present_mask |= 1u << key;
  };
  auto str = [&](int key, char* out, size_t n) {
    auto it = kv.find(kKeys[key]);
    if (it == kv.end()) return;
    if (it->second.kind != TVal::STR) { err = std::string(kKeys[key]) + ": not a string"; return; }
    std::snprintf(out, n, "%s", it->second.s.c_str());
    c->present_mask |= 1u << key;
  };
  auto integer = [&](int key, long long* out) {
    auto it = kv.find(kKeys[key]);
    if (it == kv.end()) return;
    if (it->second.kind != TVal::INT) { err = std::string(kKeys[key]) + ": not an integer"; return; }
    *out = it->second.i;
    c->present_mask |= 1u << key;
  };
  auto floating = [&](int key, float* out) {
    auto it = kv.find(kKeys[key]);
    if (it == kv.end()) return;
    if (it->second.kind != TVal::FLT) { err = std::string(kKeys[key]) + ": not a floating value"; return; }
    *out = (float)it->second.f;
    c->present_mask |= 1u << key;
  };
  long long tmp = 0;
  vec3(0, &c->look_from);
  vec3(1, &c->look_at);
  vec3(2, &c->look_up);
  floating(3, &c->fovy);
  str(4, c->photons_file, sizeof(c->photons_file));
  str(5, c->caustics_photons_file, sizeof(c->caustics_photons_file));
  str(6, c->model_path, sizeof(c->model_path));
  vec3(7, &c->sky_colour);
  str(8, c->output_filename, sizeof(c->output_filename));
  vec2i(9, &c->fb_width, &c->fb_height);
  tmp = 0; integer(10, &tmp); c->samples_per_pixel = (int32_t)tmp;
  tmp = 0; integer(11, &tmp); c->depth = (int32_t)tmp;
  str(12, c->viewer_output_filename, sizeof(c->viewer_output_filename));
  str(13, c->viewer_caustics_output_filename, sizeof(c->viewer_caustics_output_filename));
  vec2i(14, &c->viewer_fb_width, &c->viewer_fb_height);
  tmp = 0; integer(15, &tmp); c->max_depth = (int32_t)tmp;
  tmp = 0; integer(16, &tmp); c->casted_diffuse_photons = tmp;
  tmp = 0; integer(17, &tmp); c->casted_caustics_photons = tmp;
  if (!err.empty()) {
    set_err(c, err);
    return PM_ERR_INVALID;
  }
  return PM_OK;
}
