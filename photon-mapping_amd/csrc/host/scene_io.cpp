// scene_io.cpp — scene ingest for the drop-in boundary (B1).
//
// Replaces the assimp import of common/src/assetImporter.cxx:16-205 (assimp
// is not vendored: externals/assimp is empty) with an own GLB (glTF 2.0
// binary) and OBJ reader that reproduces what the reference observes:
//   * assimp's glTF2 node graph: one root (the scene's single node, or a
//     "ROOT" node over several), node matrix = T * R * S built exactly as
//     aiMatrix4x4(scaling, quaternion, position) does in float;
//   * extract_objects (assetImporter.cxx:33-96): BFS over nodes, transform =
//     node * parent (:43), per-mesh vertex de-duplication by exact position in
//     first-occurrence order (:65-73), mesh name = material name (:87-90);
//   * extract_lights (:98-134): <dir>/lights.txt, "x y z r g b power"; a line
//     "x y z r g b power nx ny nz side" is a SQUARE_LIGHT (this build's
//     extension);
//   * assign_materials (:139-205): <stem>.mtl, "name r g b d s t ior",
//     default white diffuse with ior 0.
// Deviation: the reference rewrites '/' to '\\' before
// opening lights.txt / .mtl and so cannot load a scene on Linux; both
// separators are accepted here.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <memory>
#include <iterator>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../../include/pm.h"

namespace {

// ---------------------------------------------------------------- mini JSON
struct JVal {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  double num = 0;
  bool b = false;
  std::string str;
  std::vector<JVal> arr;
  std::vector<std::pair<std::string, JVal>> obj;
  const JVal* get(const char* k) const {
    if (kind != OBJ) return nullptr;
    for (auto& kv : obj)
      if (kv.first == k) return &kv.second;
    return nullptr;
  }
  double n(const char* k, double d) const {
    const JVal* v = get(k);
    return (v && v->kind == NUM) ? v->num : d;
  }
};

struct JParser {
  const char* s;
  size_t n, p = 0;
  bool ok = true;
  void ws() { while (p < n && (s[p] == ' ' || s[p] == '\t' || s[p] == '\n' || s[p] == '\r')) p++; }
  bool parse(JVal& v) {
    ws();
    if (p >= n) return ok = false;
    char c = s[p];
    if (c == '{') {
      p++;
      v.kind = JVal::OBJ;
      ws();
      if (p < n && s[p] == '}') { p++; return true; }
      for (;;) {
        ws();
        JVal k;
        if (p >= n || s[p] != '"' || !parse(k)) return ok = false;
        ws();
        if (p >= n || s[p] != ':') return ok = false;
        p++;
        JVal val;
        if (!parse(val)) return false;
        v.obj.emplace_back(k.str, std::move(val));
        ws();
        if (p < n && s[p] == ',') { p++; continue; }
        if (p < n && s[p] == '}') { p++; return true; }
        return ok = false;
      }
    }
    if (c == '[') {
      p++;
      v.kind = JVal::ARR;
      ws();
      if (p < n && s[p] == ']') { p++; return true; }
      for (;;) {
        JVal e;
        if (!parse(e)) return false;
        v.arr.push_back(std::move(e));
        ws();
        if (p < n && s[p] == ',') { p++; continue; }
        if (p < n && s[p] == ']') { p++; return true; }
        return ok = false;
      }
    }
    if (c == '"') {
      p++;
      v.kind = JVal::STR;
      while (p < n && s[p] != '"') {
        if (s[p] == '\\' && p + 1 < n) {
          char e = s[p + 1];
          p += 2;
          if (e == 'u' && p + 4 <= n) {
            unsigned cp = (unsigned)std::strtoul(std::string(s + p, 4).c_str(), nullptr, 16);
            p += 4;
            if (cp < 0x80) v.str += (char)cp;
            else if (cp < 0x800) { v.str += (char)(0xC0 | (cp >> 6)); v.str += (char)(0x80 | (cp & 0x3F)); }
            else { v.str += (char)(0xE0 | (cp >> 12)); v.str += (char)(0x80 | ((cp >> 6) & 0x3F)); v.str += (char)(0x80 | (cp & 0x3F)); }
            continue;
          }
          switch (e) {
            case 'n': v.str += '\n'; break;
            case 't': v.str += '\t'; break;
            case 'r': v.str += '\r'; break;
            case 'b': v.str += '\b'; break;
            case 'f': v.str += '\f'; break;
            default: v.str += e; break;
          }
          continue;
        }
        v.str += s[p++];
      }
      if (p >= n) return ok = false;
      p++;
      return true;
    }
    if (!std::strncmp(s + p, "true", 4)) { p += 4; v.kind = JVal::BOOL; v.b = true; return true; }
    if (!std::strncmp(s + p, "false", 5)) { p += 5; v.kind = JVal::BOOL; return true; }
    if (!std::strncmp(s + p, "null", 4)) { p += 4; return true; }
    char* end = nullptr;
    std::string tmp(s + p, std::min<size_t>(64, n - p));
    v.num = std::strtod(tmp.c_str(), &end);
    if (end == tmp.c_str()) return ok = false;
    v.kind = JVal::NUM;
    p += (size_t)(end - tmp.c_str());
    return true;
  }
};

// -------------------------------------------------- assimp-like float matrix
struct Mat4 {  // row-major a1..d4 like aiMatrix4x4
  float m[4][4];
  static Mat4 identity() {
    Mat4 r{};
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.f;
    return r;
  }
};
// aiMatrix4x4::operator*= : this = this * other, each entry a dot of 4 terms
Mat4 mul(const Mat4& a, const Mat4& b) {
  Mat4 r{};
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 4; j++)
      r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j] + a.m[i][3] * b.m[3][j];
  return r;
}
pm_float3 xform(const Mat4& M, float x, float y, float z) {
  // aiMatrix4x4 * aiVector3D
  return {M.m[0][0] * x + M.m[0][1] * y + M.m[0][2] * z + M.m[0][3],
          M.m[1][0] * x + M.m[1][1] * y + M.m[1][2] * z + M.m[1][3],
          M.m[2][0] * x + M.m[2][1] * y + M.m[2][2] * z + M.m[2][3]};
}
// assimp glTF2Importer ImportNode: matrix, or T * R * S in that order.
Mat4 node_matrix(const JVal& node) {
  Mat4 M = Mat4::identity();
  if (const JVal* mat = node.get("matrix")) {
    if (mat->kind == JVal::ARR && mat->arr.size() == 16) {
      // glTF column-major -> row-major
      for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) M.m[r][c] = (float)mat->arr[c * 4 + r].num;
      return M;
    }
  }
  if (const JVal* t = node.get("translation")) {
    Mat4 T = Mat4::identity();
    T.m[0][3] = (float)t->arr[0].num;
    T.m[1][3] = (float)t->arr[1].num;
    T.m[2][3] = (float)t->arr[2].num;
    M = mul(M, T);
  }
  if (const JVal* q = node.get("rotation")) {
    const float x = (float)q->arr[0].num, y = (float)q->arr[1].num, z = (float)q->arr[2].num,
                w = (float)q->arr[3].num;
    Mat4 R = Mat4::identity();
    // aiQuaternion::GetMatrix
    R.m[0][0] = 1.0f - 2.0f * (y * y + z * z);
    R.m[0][1] = 2.0f * (x * y - z * w);
    R.m[0][2] = 2.0f * (x * z + y * w);
    R.m[1][0] = 2.0f * (x * y + z * w);
    R.m[1][1] = 1.0f - 2.0f * (x * x + z * z);
    R.m[1][2] = 2.0f * (y * z - x * w);
    R.m[2][0] = 2.0f * (x * z - y * w);
    R.m[2][1] = 2.0f * (y * z + x * w);
    R.m[2][2] = 1.0f - 2.0f * (x * x + y * y);
    M = mul(M, R);
  }
  if (const JVal* s = node.get("scale")) {
    Mat4 S = Mat4::identity();
    S.m[0][0] = (float)s->arr[0].num;
    S.m[1][1] = (float)s->arr[1].num;
    S.m[2][2] = (float)s->arr[2].num;
    M = mul(M, S);
  }
  return M;
}

// A mesh as assimp would hand it to extract_objects: positions + triangles.
struct RawMesh {
  std::vector<pm_float3> pos;
  std::vector<pm_int3> tris;
  std::string material;
};
struct RawNode {
  Mat4 M;
  std::vector<int> meshes;
  std::vector<int> children;
};
struct RawScene {
  std::vector<RawMesh> meshes;
  std::vector<RawNode> nodes;
  int root = 0;
};

bool read_file(const std::string& path, std::string& out) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) return false;
  std::stringstream ss;
  ss << f.rdbuf();
  out = ss.str();
  return true;
}

bool load_glb(const std::string& path, RawScene& sc, std::string& err) {
  std::string b;
  if (!read_file(path, b)) { err = "cannot open " + path; return false; }
  if (b.size() < 20) { err = "truncated glb"; return false; }
  uint32_t hdr[5];
  std::memcpy(hdr, b.data(), 20);
  if (hdr[0] != 0x46546C67u || hdr[1] != 2) { err = "not a glTF 2.0 binary"; return false; }
  const uint32_t jlen = hdr[3];
  if (hdr[4] != 0x4E4F534Au || 20 + (size_t)jlen > b.size()) { err = "bad JSON chunk"; return false; }
  JParser jp{b.data() + 20, jlen};
  JVal J;
  if (!jp.parse(J) || J.kind != JVal::OBJ) { err = "bad glTF JSON"; return false; }
  const char* bin = nullptr;
  size_t binlen = 0;
  size_t off = 20 + jlen;
  while (off + 8 <= b.size()) {
    uint32_t ch[2];
    std::memcpy(ch, b.data() + off, 8);
    if (ch[1] == 0x004E4942u) {
      bin = b.data() + off + 8;
      binlen = std::min<size_t>(ch[0], b.size() - off - 8);
      break;
    }
    off += 8 + ch[0];
  }
  const JVal* accessors = J.get("accessors");
  const JVal* views = J.get("bufferViews");
  const JVal* meshes = J.get("meshes");
  const JVal* nodes = J.get("nodes");
  const JVal* mats = J.get("materials");
  auto acc_data = [&](int ai, int& count, int& ctype, int& ncomp, const char*& base, size_t& stride) -> bool {
    if (!accessors || ai < 0 || ai >= (int)accessors->arr.size()) return false;
    const JVal& a = accessors->arr[ai];
    count = (int)a.n("count", 0);
    if (count < 0) return false;   // malformed: a negative count would skip the bounds check
    ctype = (int)a.n("componentType", 0);
    const JVal* ty = a.get("type");
    std::string t = ty ? ty->str : "";
    ncomp = t == "SCALAR" ? 1 : t == "VEC2" ? 2 : t == "VEC3" ? 3 : t == "VEC4" ? 4 : 0;
    const int bv = (int)a.n("bufferView", -1);
    if (bv < 0 || !views || bv >= (int)views->arr.size() || !bin) return false;
    const JVal& v = views->arr[bv];
    const size_t voff = (size_t)v.n("byteOffset", 0) + (size_t)a.n("byteOffset", 0);
    const int csize = (ctype == 5126 || ctype == 5125) ? 4 : (ctype == 5123 || ctype == 5122) ? 2 : 1;
    stride = (size_t)v.n("byteStride", 0);
    if (stride == 0) stride = (size_t)csize * ncomp;
    if (count > 0 && voff + stride * (size_t)(count - 1) + (size_t)csize * ncomp > binlen) return false;
    base = bin + voff;
    return true;
  };
  // meshes: one aiMesh per primitive (assimp glTF2), in mesh/primitive order
  std::vector<std::vector<int>> mesh_prims;
  if (meshes) {
    for (const JVal& m : meshes->arr) {
      std::vector<int> ids;
      const JVal* prims = m.get("primitives");
      if (prims)
        for (const JVal& pr : prims->arr) {
          const int mode = (int)pr.n("mode", 4);
          if (mode != 4) continue;   // SortByPType drops points/lines; strips unsupported
          RawMesh rm;
          const JVal* attrs = pr.get("attributes");
          const JVal* pa = attrs ? attrs->get("POSITION") : nullptr;
          int cnt, ct, nc;
          const char* base;
          size_t stride;
          if (!pa || !acc_data((int)pa->num, cnt, ct, nc, base, stride) || ct != 5126 || nc != 3) {
            err = "unsupported POSITION accessor";
            return false;
          }
          rm.pos.resize(cnt);
          for (int i = 0; i < cnt; i++) std::memcpy(&rm.pos[i], base + stride * i, 12);
          std::vector<int64_t> idx;
          const int ia = (int)pr.n("indices", -1);
          if (ia >= 0) {
            int icnt, ict, inc;
            const char* ib;
            size_t istr;
            if (!acc_data(ia, icnt, ict, inc, ib, istr) || inc != 1) { err = "bad index accessor"; return false; }
            idx.resize(icnt);
            for (int i = 0; i < icnt; i++) {
              const char* q = ib + istr * i;
              if (ict == 5125) { uint32_t v; std::memcpy(&v, q, 4); idx[i] = v; }
              else if (ict == 5123) { uint16_t v; std::memcpy(&v, q, 2); idx[i] = v; }
              else if (ict == 5121) { idx[i] = (uint8_t)*q; }
              else { err = "bad index type"; return false; }
            }
          } else {
            idx.resize(cnt);
            for (int i = 0; i < cnt; i++) idx[i] = i;
          }
          for (size_t i = 0; i + 2 < idx.size(); i += 3) {
            for (int k = 0; k < 3; k++)
              if (idx[i + k] < 0 || idx[i + k] >= cnt) { err = "index out of range"; return false; }
            rm.tris.push_back({(int32_t)idx[i], (int32_t)idx[i + 1], (int32_t)idx[i + 2]});
          }
          const int mi = (int)pr.n("material", -1);
          if (mats && mi >= 0 && mi < (int)mats->arr.size()) {
            const JVal* nm = mats->arr[mi].get("name");
            rm.material = nm ? nm->str : "";
          } else {
            rm.material = "DefaultMaterial";
          }
          ids.push_back((int)sc.meshes.size());
          sc.meshes.push_back(std::move(rm));
        }
      mesh_prims.push_back(ids);
    }
  }
  const int nn = nodes ? (int)nodes->arr.size() : 0;
  sc.nodes.resize(nn);
  for (int i = 0; i < nn; i++) {
    const JVal& nd = nodes->arr[i];
    sc.nodes[i].M = node_matrix(nd);
    const int mi = (int)nd.n("mesh", -1);
    if (mi >= 0 && mi < (int)mesh_prims.size()) sc.nodes[i].meshes = mesh_prims[mi];
    if (const JVal* ch = nd.get("children"))
      for (const JVal& c : ch->arr) sc.nodes[i].children.push_back((int)c.num);
  }
  std::vector<int> roots;
  const JVal* scenes = J.get("scenes");
  const int si = (int)J.n("scene", 0);
  if (scenes && si >= 0 && si < (int)scenes->arr.size()) {
    if (const JVal* sn = scenes->arr[si].get("nodes"))
      for (const JVal& r : sn->arr) roots.push_back((int)r.num);
  } else {
    for (int i = 0; i < nn; i++) roots.push_back(i);
  }
  if (roots.size() == 1) {
    sc.root = roots[0];
  } else {
    RawNode R;
    R.M = Mat4::identity();
    R.children = roots;
    sc.root = (int)sc.nodes.size();
    sc.nodes.push_back(R);
  }
  return true;
}

// OBJ: assimp's ObjFileImporter makes one aiMesh per (object, material)
// group; polygons are fan-triangulated here (assimp Triangulate: fan for
// convex faces). Custom-.mtl name collisions behave as upstream (§5.1-12).
bool load_obj(const std::string& path, RawScene& sc, std::string& err) {
  std::ifstream f(path);
  if (!f.is_open()) { err = "cannot open " + path; return false; }
  std::vector<pm_float3> V;
  RawNode root;
  root.M = Mat4::identity();
  std::string cur_mtl = "DefaultMaterial";
  int cur = -1;
  std::string line;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    std::string tag;
    if (!(is >> tag)) continue;
    if (tag == "v") {
      pm_float3 p{};
      is >> p.x >> p.y >> p.z;
      V.push_back(p);
    } else if (tag == "o" || tag == "g") {
      cur = -1;
    } else if (tag == "usemtl") {
      is >> cur_mtl;
      cur = -1;
    } else if (tag == "f") {
      if (cur < 0) {
        cur = (int)sc.meshes.size();
        sc.meshes.emplace_back();
        sc.meshes.back().material = cur_mtl;
        root.meshes.push_back(cur);
      }
      std::vector<int> fv;
      std::string tok;
      while (is >> tok) {
        long v = std::strtol(tok.c_str(), nullptr, 10);
        if (v < 0) v = (long)V.size() + v + 1;
        if (v < 1 || v > (long)V.size()) { err = "bad face index in " + path; return false; }
        fv.push_back((int)v - 1);
      }
      for (size_t k = 1; k + 1 < fv.size(); k++) {
        RawMesh& m = sc.meshes[cur];
        // per-mesh vertex arrays are rebuilt from global positions
        const int base = (int)m.pos.size();
        m.pos.push_back(V[fv[0]]);
        m.pos.push_back(V[fv[k]]);
        m.pos.push_back(V[fv[k + 1]]);
        m.tris.push_back({base, base + 1, base + 2});
      }
    }
  }
  sc.nodes.push_back(root);
  sc.root = 0;
  return true;
}

std::string dir_of(const std::string& path) {
  const size_t s = path.find_last_of("/\\");
  return s == std::string::npos ? std::string(".") : path.substr(0, s);
}
std::string stem_of(const std::string& path) {
  const size_t d = path.find_last_of('.');
  const size_t s = path.find_last_of("/\\");
  if (d == std::string::npos || (s != std::string::npos && d < s)) return path;
  return path.substr(0, d);
}
std::string native(std::string p) {
  for (char& c : p)
    if (c == '\\') c = '/';
  return p;
}

}  // namespace

struct pm_scene_data {
  std::vector<std::vector<pm_float3>> verts;
  std::vector<std::vector<pm_int3>> idx;
  std::vector<std::string> names;
  std::vector<pm_mesh> meshes;
  std::vector<pm_light> lights;
  int64_t nv = 0, nt = 0;
};

extern "C" int pm_scene_data_load(const char* cpath, pm_scene_data** out) {
  if (!cpath || !out) return PM_ERR_INVALID;
  *out = nullptr;
  const std::string path = native(cpath);
  RawScene sc;
  std::string err;
  std::string ext = path.size() >= 4 ? path.substr(path.size() - 4) : "";
  for (char& c : ext) c = (char)std::tolower((unsigned char)c);
  bool ok = ext == ".obj" ? load_obj(path, sc, err) : load_glb(path, sc, err);
  if (!ok) {
    std::fprintf(stderr, "pm: scene import failed: %s\n", err.c_str());
    return PM_ERR_IO;
  }
  std::unique_ptr<pm_scene_data> S(new pm_scene_data);
  // extract_objects: BFS, transform = node * parent
  // glTF node graphs are trees: a node reached twice (a cycle, or two parents)
  // is malformed and rejected instead of looping forever
  std::deque<std::pair<int, Mat4>> q;
  std::vector<char> seen(sc.nodes.size(), 0);
  q.emplace_back(sc.root, Mat4::identity());
  while (!q.empty()) {
    auto [ni, parent] = q.front();
    q.pop_front();
    if (ni < 0 || ni >= (int)sc.nodes.size()) continue;
    if (seen[ni]) {
      std::fprintf(stderr, "pm: scene import failed: node %d is reached twice (cyclic node hierarchy)\n", ni);
      return PM_ERR_IO;
    }
    seen[ni] = 1;
    const RawNode& node = sc.nodes[ni];
    const Mat4 T = mul(node.M, parent);
    for (int c : node.children) q.emplace_back(c, T);
    for (int mi : node.meshes) {
      if (mi < 0 || mi >= (int)sc.meshes.size()) {
        std::fprintf(stderr, "pm: scene import failed: node %d names mesh %d of %zu\n", ni, mi, sc.meshes.size());
        return PM_ERR_IO;
      }
      const RawMesh& rm = sc.meshes[mi];
      std::vector<pm_float3> verts;
      std::vector<pm_int3> idx;
      // exact-position dedup in first-occurrence order (std::find semantics)
      std::unordered_map<uint64_t, std::vector<int>> buckets;
      auto find_or_add = [&](pm_float3 p) -> int {
        uint32_t bx, by, bz;
        std::memcpy(&bx, &p.x, 4); std::memcpy(&by, &p.y, 4); std::memcpy(&bz, &p.z, 4);
        // hash on value class (+0 == -0 compare equal under operator==)
        auto canon = [](uint32_t u) { return (u == 0x80000000u) ? 0u : u; };
        const uint64_t h = (uint64_t)canon(bx) * 0x9E3779B97F4A7C15ull ^ (uint64_t)canon(by) * 0xC2B2AE3D27D4EB4Full ^
                           (uint64_t)canon(bz);
        auto& bk = buckets[h];
        for (int j : bk)
          if (verts[j].x == p.x && verts[j].y == p.y && verts[j].z == p.z) return j;
        verts.push_back(p);
        bk.push_back((int)verts.size() - 1);
        return (int)verts.size() - 1;
      };
      for (const pm_int3& t : rm.tris) {
        const int a = find_or_add(xform(T, rm.pos[t.x].x, rm.pos[t.x].y, rm.pos[t.x].z));
        const int b = find_or_add(xform(T, rm.pos[t.y].x, rm.pos[t.y].y, rm.pos[t.y].z));
        const int c = find_or_add(xform(T, rm.pos[t.z].x, rm.pos[t.z].y, rm.pos[t.z].z));
        idx.push_back({a, b, c});
      }
      S->verts.push_back(std::move(verts));
      S->idx.push_back(std::move(idx));
      S->names.push_back(rm.material);
    }
  }
  // extract_lights
  {
    const std::string lp = dir_of(path) + "/lights.txt";
    std::ifstream lf(lp);
    if (!lf.is_open()) {
      std::fprintf(stderr, "pm: Unable to open file: %s\n", lp.c_str());
      return PM_ERR_IO;
    }
    std::string line;
    while (std::getline(lf, line)) {
      if (line.empty() || line[0] == '#') continue;
      std::istringstream is(line);
      pm_light L;
      std::memset(&L, 0, sizeof(L));
      L.source_type = PM_POINT_LIGHT;
      if (!(is >> L.pos.x >> L.pos.y >> L.pos.z >> L.rgb.x >> L.rgb.y >> L.rgb.z >> L.power)) {
        std::fprintf(stderr, "pm: Invalid light source data format\n");
        return PM_ERR_IO;
      }
      // extension (this build): "... power nx ny nz side" = SQUARE_LIGHT
      std::string extra;
      if (is >> extra) {
        std::istringstream rest(extra + " " + std::string(std::istreambuf_iterator<char>(is), {}));
        double side = 0;
        if (!(rest >> L.normal.x >> L.normal.y >> L.normal.z >> side)) {
          std::fprintf(stderr, "pm: Invalid light source data format\n");
          return PM_ERR_IO;
        }
        L.source_type = PM_SQUARE_LIGHT;
        L.side_length = side;
      }
      S->lights.push_back(L);
    }
  }
  // assign_materials
  std::map<std::string, pm_material> mm;
  {
    const std::string mp = stem_of(path) + ".mtl";
    std::ifstream mf(mp);
    if (!mf.is_open()) {
      std::fprintf(stderr, "Error: Unable to open file %s\n", mp.c_str());
    } else {
      std::string line;
      while (std::getline(mf, line)) {
        if (line.empty() || line[0] == '#') continue;
        std::istringstream is(line);
        std::string name;
        pm_material m;
        if (is >> name >> m.albedo.x >> m.albedo.y >> m.albedo.z >> m.diffuse >> m.specular >> m.transmission >>
            m.refraction_idx) {
          mm[name] = m;
        } else {
          std::fprintf(stderr, "Warning: Invalid line format: %s\n", line.c_str());
        }
      }
    }
  }
  const pm_material def = {{1.f, 1.f, 1.f}, 1.f, 0.f, 0.f, 0.f};
  for (size_t i = 0; i < S->verts.size(); i++) {
    pm_mesh m;
    m.vertices = S->verts[i].data();
    m.num_vertices = (int32_t)S->verts[i].size();
    m.indices = S->idx[i].data();
    m.num_triangles = (int32_t)S->idx[i].size();
    auto it = mm.find(S->names[i]);
    m.material = it == mm.end() ? def : it->second;
    S->meshes.push_back(m);
    S->nv += m.num_vertices;
    S->nt += m.num_triangles;
  }
  *out = S.release();
  return PM_OK;
}

extern "C" int pm_scene_data_counts(const pm_scene_data* s, int32_t* nm, int32_t* nl, int64_t* nv, int64_t* nt) {
  if (!s) return PM_ERR_INVALID;
  if (nm) *nm = (int32_t)s->meshes.size();
  if (nl) *nl = (int32_t)s->lights.size();
  if (nv) *nv = s->nv;
  if (nt) *nt = s->nt;
  return PM_OK;
}
extern "C" int pm_scene_data_meshes(const pm_scene_data* s, const pm_mesh** m) {
  if (!s || !m) return PM_ERR_INVALID;
  *m = s->meshes.data();
  return PM_OK;
}
extern "C" int pm_scene_data_lights(const pm_scene_data* s, const pm_light** l) {
  if (!s || !l) return PM_ERR_INVALID;
  *l = s->lights.data();
  return PM_OK;
}
extern "C" int pm_scene_data_mesh_name(const pm_scene_data* s, int32_t i, const char** name) {
  if (!s || !name || i < 0 || i >= (int32_t)s->names.size()) return PM_ERR_INVALID;
  *name = s->names[i].c_str();
  return PM_OK;
}
extern "C" int pm_scene_data_free(pm_scene_data* s) {
  delete s;
  return PM_OK;
}
