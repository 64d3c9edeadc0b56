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
#include <algorithm>
#include <array>
#include <cmath>
#include <functional>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <deque>
#include <fstream>
#include <map>
#include <set>
#include <memory>
#include <iterator>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include <zlib.h>

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

// ------------------------------------------------------------------ FBX
// Binary FBX (7100-7500; the reference's assets/models/cornell-box/cornell-box.fbx
// is 7400, reached through assimp at assetImporter.cxx:18-21). What assimp's
// FBX importer (+ Triangulate) hands extract_objects, restated:
//   * nodes: a root over the models connected to object 0 (connection order),
//     each model's children likewise; the model matrix is T * R * S in float
//     (aiMatrix4x4 products), R = Rz * Ry * Rx of the Euler angles in degrees
//     (rotation order XYZ). Pivots, offsets, pre/post and geometric transforms
//     would make assimp insert helper nodes: rejected here (none in the assets);
//   * meshes: one per (geometry, material index) in first-appearance order,
//     vertices = polygon corners (positions cast from double), named after the
//     model's connected material ("DefaultMaterial" when none);
//   * Triangulate: quads split from the first vertex whose two angles to the
//     diagonal exceed pi (assimp's concave-quad rule), larger polygons as a fan.
// Parity for FBX is unpinned: assimp cannot be run here; tests compare the
// scene against the same model's GLB.
struct FbxProp {
  char type = 0;
  double num = 0.0;      // scalar types
  int64_t inum = 0;
  std::string str;       // S / R
  std::vector<double> darr;   // f / d arrays
  std::vector<int64_t> iarr;  // i / l / b arrays
};
struct FbxNode {
  std::string name;
  std::vector<FbxProp> props;
  std::vector<FbxNode> kids;
  const FbxNode* child(const char* n) const {
    for (const FbxNode& k : kids)
      if (k.name == n) return &k;
    return nullptr;
  }
};

struct FbxReader {
  const std::string& b;
  bool wide = false;
  std::string err;
  template <typename T>
  bool rd(size_t o, T& v) {
    if (o + sizeof(T) > b.size()) return false;
    std::memcpy(&v, b.data() + o, sizeof(T));
    return true;
  }
  bool array(size_t& p, char t, FbxProp& pr) {
    uint32_t n = 0, enc = 0, clen = 0;
    if (!rd(p, n) || !rd(p + 4, enc) || !rd(p + 8, clen) || p + 12 + (size_t)clen > b.size()) return false;
    p += 12;
    const size_t es = (t == 'd' || t == 'l') ? 8 : (t == 'b' ? 1 : 4);
    std::string raw;
    if (enc == 0) {
      if ((size_t)n * es != clen) return false;
      raw.assign(b.data() + p, clen);
    } else if (enc == 1) {
      // zlib cannot expand by more than ~1032:1: a header asking for more is
      // malformed (and would otherwise allocate up to 32 GB from a tiny file)
      if ((size_t)n * es > (size_t)clen * 1032 + 64) return false;
      raw.resize((size_t)n * es);
      uLongf dl = (uLongf)raw.size();
      if (uncompress((Bytef*)&raw[0], &dl, (const Bytef*)b.data() + p, clen) != Z_OK || dl != raw.size()) return false;
    } else {
      return false;
    }
    p += clen;
    for (uint32_t i = 0; i < n; i++) {
      const char* q = raw.data() + (size_t)i * es;
      if (t == 'd') { double v; std::memcpy(&v, q, 8); pr.darr.push_back(v); }
      else if (t == 'f') { float v; std::memcpy(&v, q, 4); pr.darr.push_back(v); }
      else if (t == 'l') { int64_t v; std::memcpy(&v, q, 8); pr.iarr.push_back(v); }
      else if (t == 'i') { int32_t v; std::memcpy(&v, q, 4); pr.iarr.push_back(v); }
      else pr.iarr.push_back(*q ? 1 : 0);
    }
    return true;
  }
  // one node record at o; false on a malformed record; `null` for the end marker
  bool node(size_t& o, FbxNode& out, bool& null, int depth) {
    uint64_t end = 0, nprop = 0, plen = 0;
    if (wide) {
      if (!rd(o, end) || !rd(o + 8, nprop) || !rd(o + 16, plen)) return false;
      o += 24;
    } else {
      uint32_t e32, n32, p32;
      if (!rd(o, e32) || !rd(o + 4, n32) || !rd(o + 8, p32)) return false;
      end = e32, nprop = n32, plen = p32;
      o += 12;
    }
    uint8_t nl = 0;
    if (!rd(o, nl)) return false;
    o += 1;
    null = end == 0;
    if (null) return true;
    if (end > b.size() || o + nl > end || depth > 64) return false;
    out.name.assign(b.data() + o, nl);
    o += nl;
    size_t p = o;
    for (uint64_t k = 0; k < nprop; k++) {
      FbxProp pr;
      if (p >= end) return false;
      pr.type = b[p++];
      switch (pr.type) {
        case 'Y': { int16_t v; if (!rd(p, v)) return false; pr.inum = v; pr.num = v; p += 2; break; }
        case 'C': { uint8_t v; if (!rd(p, v)) return false; pr.inum = v; pr.num = v; p += 1; break; }
        case 'I': { int32_t v; if (!rd(p, v)) return false; pr.inum = v; pr.num = v; p += 4; break; }
        case 'F': { float v; if (!rd(p, v)) return false; pr.num = v; pr.inum = (int64_t)v; p += 4; break; }
        case 'D': { double v; if (!rd(p, v)) return false; pr.num = v; pr.inum = (int64_t)v; p += 8; break; }
        case 'L': { int64_t v; if (!rd(p, v)) return false; pr.inum = v; pr.num = (double)v; p += 8; break; }
        case 'f': case 'd': case 'l': case 'i': case 'b':
          if (!array(p, pr.type, pr)) return false;
          break;
        case 'S': case 'R': {
          uint32_t n; if (!rd(p, n) || p + 4 + (size_t)n > end) return false;
          pr.str.assign(b.data() + p + 4, n);
          p += 4 + n;
          break;
        }
        default:
          return false;
      }
      out.props.push_back(std::move(pr));
    }
    o = p;
    while (o < end) {
      FbxNode kid;
      bool kn = false;
      if (!node(o, kid, kn, depth + 1)) return false;
      if (kn) break;
      out.kids.push_back(std::move(kid));
    }
    o = (size_t)end;
    return true;
  }
};

// "name\0\1Class" -> name
std::string fbx_name(const std::string& s) {
  const size_t z = s.find('\0');
  return z == std::string::npos ? s : s.substr(0, z);
}

// Properties70 P records of a model: name -> values (doubles)
std::map<std::string, std::vector<double>> fbx_p70(const FbxNode& obj) {
  std::map<std::string, std::vector<double>> out;
  const FbxNode* p70 = obj.child("Properties70");
  if (!p70) return out;
  for (const FbxNode& p : p70->kids) {
    if (p.name != "P" || p.props.empty()) continue;
    std::vector<double> v;
    for (size_t i = 4; i < p.props.size(); i++) v.push_back(p.props[i].num);
    out[p.props[0].str] = v;
  }
  return out;
}

// aiMatrix4x4::RotationX / Y / Z (angle in radians, float)
Mat4 rot_axis(int axis, float a) {
  Mat4 R = Mat4::identity();
  const float c = std::cos(a), s = std::sin(a);
  const int i = (axis + 1) % 3, j = (axis + 2) % 3;
  R.m[i][i] = c;
  R.m[i][j] = -s;
  R.m[j][i] = s;
  R.m[j][j] = c;
  return R;
}

bool load_fbx(const std::string& path, RawScene& sc, std::string& err) {
  std::string b;
  if (!read_file(path, b)) { err = "cannot open " + path; return false; }
  static const char magic[] = "Kaydara FBX Binary  ";
  if (b.size() < 27 || std::memcmp(b.data(), magic, 20) != 0) {
    err = "not a binary FBX (ASCII FBX is not supported)";
    return false;
  }
  uint32_t ver = 0;
  std::memcpy(&ver, b.data() + 23, 4);
  FbxReader R{b};
  R.wide = ver >= 7500;
  std::vector<FbxNode> top;
  size_t o = 27;
  while (o < b.size()) {
    FbxNode nd;
    bool null = false;
    if (!R.node(o, nd, null, 0)) { err = "malformed FBX record"; return false; }
    if (null) break;
    top.push_back(std::move(nd));
  }
  const FbxNode* objects = nullptr;
  const FbxNode* conns = nullptr;
  for (const FbxNode& n : top) {
    if (n.name == "Objects") objects = &n;
    if (n.name == "Connections") conns = &n;
  }
  if (!objects || !conns) { err = "FBX without Objects / Connections"; return false; }
  std::map<int64_t, const FbxNode*> geoms, models, mats;
  for (const FbxNode& ob : objects->kids) {
    if (ob.props.empty()) continue;
    const int64_t id = ob.props[0].inum;
    if (ob.name == "Geometry" && ob.props.size() >= 3 && ob.props[2].str == "Mesh") geoms[id] = &ob;
    else if (ob.name == "Model") models[id] = &ob;
    else if (ob.name == "Material") mats[id] = &ob;
  }
  // object-object connections in file order: child -> parent
  std::vector<std::pair<int64_t, int64_t>> oo;
  for (const FbxNode& c : conns->kids)
    if (c.name == "C" && c.props.size() >= 3 && c.props[0].str == "OO") oo.push_back({c.props[1].inum, c.props[2].inum});
  // model -> its geometries / materials / child models, in connection order
  std::map<int64_t, std::vector<int64_t>> mgeo, mmat, mkids;
  std::vector<int64_t> roots;
  std::map<int64_t, int64_t> parent_of;
  for (const auto& [ch, par] : oo) {
    if (geoms.count(ch) && models.count(par)) mgeo[par].push_back(ch);
    else if (mats.count(ch) && models.count(par)) mmat[par].push_back(ch);
    else if (models.count(ch)) {
      if (par != 0 && !models.count(par)) continue;
      // a node hierarchy is a tree (as load_glb requires): one parent per
      // model; the same child -> parent connection repeated is one edge
      const auto it = parent_of.find(ch);
      if (it != parent_of.end()) {
        if (it->second == par) continue;
        err = "FBX model " + std::to_string(ch) + " has two parents";
        return false;
      }
      parent_of[ch] = par;
      if (par == 0) roots.push_back(ch);
      else mkids[par].push_back(ch);
    }
  }
  static const char* complex[] = {"RotationOffset", "RotationPivot", "PreRotation", "PostRotation", "ScalingOffset",
                                  "ScalingPivot", "GeometricTranslation", "GeometricRotation", "GeometricScaling"};
  std::map<int64_t, int> node_of;
  std::set<int64_t> on_path;   // models being built: reaching one again is a cycle
  std::function<int(int64_t)> build_node = [&](int64_t id) -> int {
    if (!on_path.insert(id).second || node_of.count(id)) {
      err = "FBX model hierarchy has a cycle through model " + std::to_string(id);
      return -1;
    }
    const FbxNode& m = *models.at(id);
    const auto P = fbx_p70(m);
    for (const char* c : complex) {
      auto it = P.find(c);
      if (it == P.end()) continue;
      const double idv = std::string(c).find("Scaling") != std::string::npos && std::string(c).find("Geometric") == 0
                             ? 1.0 : 0.0;
      for (double v : it->second)
        if (v != idv) { err = std::string("FBX transform component not supported: ") + c; return -1; }
    }
    auto ro = P.find("RotationOrder");
    if (ro != P.end() && !ro->second.empty() && ro->second[0] != 0.0) { err = "FBX rotation order not XYZ"; return -1; }
    RawNode nd;
    nd.M = Mat4::identity();
    auto vec = [&](const char* k, float d) {
      auto it = P.find(k);
      std::array<float, 3> v{d, d, d};
      if (it != P.end() && it->second.size() >= 3)
        for (int i = 0; i < 3; i++) v[i] = (float)it->second[i];
      return v;
    };
    const auto t = vec("Lcl Translation", 0.f), r = vec("Lcl Rotation", 0.f), s = vec("Lcl Scaling", 1.f);
    Mat4 T = Mat4::identity();
    T.m[0][3] = t[0], T.m[1][3] = t[1], T.m[2][3] = t[2];
    const float d2r = (float)(3.14159265358979323846 / 180.0);
    Mat4 Rm = Mat4::identity();
    if (r[0] != 0.f || r[1] != 0.f || r[2] != 0.f)
      Rm = mul(mul(rot_axis(2, r[2] * d2r), rot_axis(1, r[1] * d2r)), rot_axis(0, r[0] * d2r));
    Mat4 S = Mat4::identity();
    S.m[0][0] = s[0], S.m[1][1] = s[1], S.m[2][2] = s[2];
    nd.M = mul(mul(mul(nd.M, T), Rm), S);
    // meshes: per geometry, per material index in first-appearance order
    for (int64_t gid : mgeo[id]) {
      const FbxNode& g = *geoms.at(gid);
      const FbxNode* vn = g.child("Vertices");
      const FbxNode* pn = g.child("PolygonVertexIndex");
      if (!vn || !pn || vn->props.empty() || pn->props.empty()) { err = "FBX mesh without vertices"; return -1; }
      const std::vector<double>& V = vn->props[0].darr;
      const std::vector<int64_t>& PI = pn->props[0].iarr;
      std::vector<std::vector<int>> polys;
      std::vector<int> cur;
      for (int64_t x : PI) {
        const int64_t v = x < 0 ? ~x : x;
        if (v < 0 || 3 * v + 2 >= (int64_t)V.size()) { err = "FBX polygon index out of range"; return -1; }
        cur.push_back((int)v);
        if (x < 0) {
          polys.push_back(cur);
          cur.clear();
        }
      }
      std::vector<int> pmat(polys.size(), 0);
      if (const FbxNode* lm = g.child("LayerElementMaterial")) {
        const FbxNode* mp = lm->child("MappingInformationType");
        const FbxNode* mi = lm->child("Materials");
        if (mp && mi && !mp->props.empty() && !mi->props.empty()) {
          const auto& idx = mi->props[0].iarr;
          if (mp->props[0].str == "ByPolygon") {
            for (size_t k = 0; k < polys.size() && k < idx.size(); k++) pmat[k] = (int)idx[k];
          } else if (!idx.empty()) {
            std::fill(pmat.begin(), pmat.end(), (int)idx[0]);
          }
        }
      }
      std::vector<int> order;
      for (int mi : pmat)
        if (std::find(order.begin(), order.end(), mi) == order.end()) order.push_back(mi);
      for (int mi : order) {
        RawMesh rm;
        const auto& ml = mmat[id];
        const FbxNode* mat = (mi >= 0 && mi < (int)ml.size()) ? mats.at(ml[mi]) : nullptr;
        rm.material = mat && mat->props.size() >= 2 ? fbx_name(mat->props[1].str) : "DefaultMaterial";
        for (size_t k = 0; k < polys.size(); k++) {
          if (pmat[k] != mi || polys[k].size() < 3) continue;
          const int base = (int)rm.pos.size();
          for (int v : polys[k]) rm.pos.push_back({(float)V[3 * v], (float)V[3 * v + 1], (float)V[3 * v + 2]});
          const int n = (int)polys[k].size();
          if (n == 3) {
            rm.tris.push_back({base, base + 1, base + 2});
          } else if (n == 4) {   // assimp Triangulate: start at a concave corner, if any
            int sv = 0;
            for (int i = 0; i < 4; i++) {
              auto P3 = [&](int c) { return rm.pos[base + c]; };
              const pm_float3 v = P3(i), v0 = P3((i + 3) % 4), v1 = P3((i + 2) % 4), v2 = P3((i + 1) % 4);
              auto sub = [](pm_float3 a, pm_float3 c) { return pm_float3{a.x - c.x, a.y - c.y, a.z - c.z}; };
              auto nrm = [](pm_float3 a) {
                const float l = std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z);
                return l > 0.f ? pm_float3{a.x / l, a.y / l, a.z / l} : a;
              };
              auto dot = [](pm_float3 a, pm_float3 c) { return a.x * c.x + a.y * c.y + a.z * c.z; };
              const pm_float3 left = nrm(sub(v0, v)), diag = nrm(sub(v1, v)), right = nrm(sub(v2, v));
              const float ang = std::acos(dot(left, diag)) + std::acos(dot(right, diag));
              if (ang > 3.14159265358979f) { sv = i; break; }
            }
            rm.tris.push_back({base + sv, base + (sv + 1) % 4, base + (sv + 2) % 4});
            rm.tris.push_back({base + sv, base + (sv + 2) % 4, base + (sv + 3) % 4});
          } else {
            for (int k2 = 1; k2 + 1 < n; k2++) rm.tris.push_back({base, base + k2, base + k2 + 1});
          }
        }
        nd.meshes.push_back((int)sc.meshes.size());
        sc.meshes.push_back(std::move(rm));
      }
    }
    const int me = (int)sc.nodes.size();
    sc.nodes.push_back(nd);
    node_of[id] = me;
    for (int64_t k : mkids[id]) {
      const int c = build_node(k);
      if (c < 0) return -1;
      sc.nodes[me].children.push_back(c);
    }
    on_path.erase(id);
    return me;
  };
  RawNode root;
  root.M = Mat4::identity();
  sc.nodes.push_back(root);
  sc.root = 0;
  for (int64_t r : roots) {
    const int c = build_node(r);
    if (c < 0) return false;
    sc.nodes[0].children.push_back(c);
  }
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

static int scene_data_load(const char* cpath, pm_scene_data** out);

// No C++ exception crosses the C ABI: an allocation failure or a malformed file
// that a parser step did not anticipate becomes PM_ERR_IO.
extern "C" int pm_scene_data_load(const char* cpath, pm_scene_data** out) {
  try {
    return scene_data_load(cpath, out);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "pm: scene import failed: %s\n", e.what());
  } catch (...) {
    std::fprintf(stderr, "pm: scene import failed: unknown error\n");
  }
  if (out) *out = nullptr;
  return PM_ERR_IO;
}

static int scene_data_load(const char* cpath, pm_scene_data** out) {
  if (!cpath || !out) return PM_ERR_INVALID;
  *out = nullptr;
  const std::string path = native(cpath);
  RawScene sc;
  std::string err;
  std::string ext = path.size() >= 4 ? path.substr(path.size() - 4) : "";
  for (char& c : ext) c = (char)std::tolower((unsigned char)c);
  bool ok = ext == ".obj" ? load_obj(path, sc, err) : ext == ".fbx" ? load_fbx(path, sc, err) : load_glb(path, sc, err);
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
