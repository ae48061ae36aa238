// Native tensor-tree codec for the actor <-> inference-server <-> learner data plane (utils/serialize.py).
//
// The frame format is the Python codec's, unchanged (so frames from either side interoperate and the learner's
// trajectory ring keeps parsing headers with json):
//     "ASTR1" | u64 header_len | u8 compressed | JSON header | zero pad to 64 | body (tensor bytes, 64-B aligned)
// with header nodes {"__d__": [[key, node], ...]}, {"__l__": [...]}, {"__tu__": [...]},
// {"__t__": [dtype, shape, body_offset, nbytes]}, {"__v__": scalar}.
//
// Why native: an agent step's request is a tree of ~120 small tensors and a trajectory ~64 x 150.  The Python
// encoder spends ~10 us per tensor leaf in attribute calls (detach / contiguous / view / numpy / slice
// assignment) - 3 ms per request and ~380 ms per trajectory (tools/actor_step_profile.py), which made the env
// workers, and on the server side the request decode, the pipeline's bottleneck.  Here a leaf is a type check,
// a pointer read and one memcpy; the header is emitted and parsed without building intermediate JSON objects.
// Reference counterpart: the reference pickles + lz4-compresses every trajectory (file_helper.py:255-302).
#include <torch/extension.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

constexpr char kMagic[] = "ASTR1";
constexpr size_t kMagicLen = 5;
constexpr int64_t kAlign = 64;

const char* dtype_code(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return "f32";
    case at::kHalf: return "f16";
    case at::kBFloat16: return "bf16";
    case at::kDouble: return "f64";
    case at::kLong: return "i64";
    case at::kInt: return "i32";
    case at::kShort: return "i16";
    case at::kChar: return "i8";
    case at::kByte: return "u8";
    case at::kBool: return "b";
    default: return nullptr;
  }
}

bool dtype_from_code(const std::string& s, at::ScalarType* t) {
  static const std::pair<const char*, at::ScalarType> tab[] = {
      {"f32", at::kFloat}, {"f16", at::kHalf}, {"bf16", at::kBFloat16}, {"f64", at::kDouble}, {"i64", at::kLong},
      {"i32", at::kInt},   {"i16", at::kShort}, {"i8", at::kChar},       {"u8", at::kByte},    {"b", at::kBool}};
  for (const auto& e : tab)
    if (s == e.first) {
      *t = e.second;
      return true;
    }
  return false;
}

void json_string(std::string& out, const char* s, size_t n) {
  out.push_back('"');
  for (size_t i = 0; i < n; ++i) {
    const unsigned char c = static_cast<unsigned char>(s[i]);
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      default:
        if (c < 0x20) {
          char buf[8];
          snprintf(buf, sizeof(buf), "\\u%04x", c);
          out += buf;
        } else if (c < 0x80) {
          out.push_back(static_cast<char>(c));
        } else {   // non-ASCII: \uXXXX (surrogate pairs above the BMP), as json.dumps(ensure_ascii=True)
          unsigned cp = 0;
          int extra = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : 1;
          cp = c & (0x3F >> extra);
          for (int k = 0; k < extra && i + 1 < n; ++k) cp = (cp << 6) | (static_cast<unsigned char>(s[++i]) & 0x3F);
          char buf[16];
          if (cp >= 0x10000) {
            cp -= 0x10000;
            snprintf(buf, sizeof(buf), "\\u%04x\\u%04x", 0xD800 + (cp >> 10), 0xDC00 + (cp & 0x3FF));
          } else {
            snprintf(buf, sizeof(buf), "\\u%04x", cp);
          }
          out += buf;
        }
    }
  }
  out.push_back('"');
}

void json_double(std::string& out, double v) {
  if (std::isnan(v)) { out += "NaN"; return; }
  if (std::isinf(v)) { out += v > 0 ? "Infinity" : "-Infinity"; return; }
  char buf[40];
  snprintf(buf, sizeof(buf), "%.17g", v);
  out += buf;
  // keep it a float on the way back ("1" would decode as an int)
  if (!strpbrk(buf, ".eEn")) out += ".0";
}

using Trims = std::map<std::string, std::vector<std::pair<int64_t, std::vector<int64_t>>>>;

struct Encoder {
  std::string header;
  std::vector<std::pair<int64_t, at::Tensor>> blobs;
  int64_t offset = 0;
  // row mode (rows_dumps): every tensor leaf with a batch dim becomes leaf[row], narrowed per `trims`
  int64_t row = -1;
  const Trims* trims = nullptr;
  std::string path;

  void scalar(py::handle o) {
    header += "{\"__v__\": ";
    if (o.is_none()) {
      header += "null";
    } else if (PyBool_Check(o.ptr())) {
      header += o.ptr() == Py_True ? "true" : "false";
    } else if (PyLong_Check(o.ptr())) {
      int overflow = 0;
      const long long v = PyLong_AsLongLongAndOverflow(o.ptr(), &overflow);
      if (overflow) {
        header += py::str(o).cast<std::string>();
      } else {
        header += std::to_string(v);
      }
    } else if (PyFloat_Check(o.ptr())) {
      const double v = PyFloat_AsDouble(o.ptr());
      if (std::isfinite(v)) {
        header += py::repr(o).cast<std::string>();   // shortest round-trip form, as json.dumps
      } else {
        json_double(header, v);
      }
    } else {   // str
      Py_ssize_t n = 0;
      const char* s = PyUnicode_AsUTF8AndSize(o.ptr(), &n);
      if (!s) throw py::error_already_set();
      json_string(header, s, static_cast<size_t>(n));
    }
    header += "}";
  }

  void tensor(const at::Tensor& t0) {
    at::Tensor t = t0.is_cpu() ? t0 : t0.cpu();
    t = t.contiguous();
    const char* code = dtype_code(t.scalar_type());
    if (!code) throw py::type_error("tree_dumps: unsupported tensor dtype");
    const int64_t off = (offset + kAlign - 1) / kAlign * kAlign;
    const int64_t nbytes = t.numel() * static_cast<int64_t>(t.element_size());
    blobs.emplace_back(off, t);
    offset = off + nbytes;
    header += "{\"__t__\": [\"";
    header += code;
    header += "\", [";
    for (int64_t d = 0; d < t.dim(); ++d) {
      if (d) header += ", ";
      header += std::to_string(t.size(d));
    }
    header += "], ";
    header += std::to_string(off);
    header += ", ";
    header += std::to_string(nbytes);
    header += "]}";
  }

  at::Tensor row_view(const at::Tensor& t0) const {
    if (t0.dim() == 0) return t0;
    at::Tensor t = t0.select(0, row);
    if (trims) {
      auto it = trims->find(path);
      if (it != trims->end())
        for (const auto& dl : it->second) {
          const int64_t d = dl.first, len = dl.second[static_cast<size_t>(row)];
          if (d < t.dim()) t = t.narrow(d, 0, std::max<int64_t>(0, std::min(len, t.size(d))));
        }
    }
    return t;
  }

  void node(py::handle o) {
    PyObject* p = o.ptr();
    if (THPVariable_Check(p)) {
      tensor(row >= 0 ? row_view(THPVariable_Unpack(p)) : THPVariable_Unpack(p));
    } else if (PyDict_Check(p)) {
      header += "{\"__d__\": [";
      PyObject *k, *v;
      Py_ssize_t pos = 0;
      bool first = true;
      while (PyDict_Next(p, &pos, &k, &v)) {
        if (!first) header += ", ";
        first = false;
        header += "[";
        if (PyUnicode_Check(k)) {
          Py_ssize_t n = 0;
          const char* s = PyUnicode_AsUTF8AndSize(k, &n);
          if (!s) throw py::error_already_set();
          json_string(header, s, static_cast<size_t>(n));
        } else if (PyLong_Check(k) && !PyBool_Check(k)) {
          header += py::str(k).cast<std::string>();   // [key, node] pairs keep int keys ints
        } else {
          throw py::type_error("tree_dumps: dict keys must be str or int");
        }
        header += ", ";
        if (row >= 0) {
          const size_t keep = path.size();
          if (!path.empty()) path += '/';
          path += py::str(k).cast<std::string>();
          node(v);
          path.resize(keep);
        } else {
          node(v);
        }
        header += "]";
      }
      header += "]}";
    } else if (PyList_Check(p) || PyTuple_Check(p)) {
      const bool is_list = PyList_Check(p);
      header += is_list ? "{\"__l__\": [" : "{\"__tu__\": [";
      const Py_ssize_t n = is_list ? PyList_GET_SIZE(p) : PyTuple_GET_SIZE(p);
      for (Py_ssize_t i = 0; i < n; ++i) {
        if (i) header += ", ";
        node(is_list ? PyList_GET_ITEM(p, i) : PyTuple_GET_ITEM(p, i));
      }
      header += "]}";
    } else if (p == Py_None || PyBool_Check(p) || PyLong_Check(p) || PyFloat_Check(p) || PyUnicode_Check(p)) {
      scalar(o);
    } else {
      // numpy arrays / numpy scalars and anything else: the Python codec handles them
      throw py::type_error("tree_dumps: unsupported leaf type");
    }
  }
};

// ------------------------------------------------------------------------------------------------- decode
struct Decoder {
  const char* s;
  const char* end;
  const uint8_t* body;
  int64_t body_len;
  bool copy;
  py::object owner;    // keeps the source buffer alive for aliasing (copy=False) tensors

  [[noreturn]] void fail(const char* what) const { throw py::value_error(std::string("tree_loads: ") + what); }

  void ws() {
    while (s < end && (*s == ' ' || *s == '\n' || *s == '\r' || *s == '\t')) ++s;
  }
  void expect(char c) {
    ws();
    if (s >= end || *s != c) fail("malformed header");
    ++s;
  }
  bool peek(char c) {
    ws();
    return s < end && *s == c;
  }

  unsigned hex4(const char* p) const {
    unsigned v = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = p[i];
      const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
      if (d < 0) fail("bad \\u escape");
      v = v * 16 + static_cast<unsigned>(d);
    }
    return v;
  }

  std::string str() {
    expect('"');
    std::string out;
    while (s < end && *s != '"') {
      char c = *s++;
      if (c != '\\') {
        out.push_back(c);
        continue;
      }
      if (s >= end) fail("bad escape");
      c = *s++;
      switch (c) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          if (end - s < 4) fail("bad \\u escape");
          unsigned cp = hex4(s);
          s += 4;
          if (cp >= 0xD800 && cp < 0xDC00 && end - s >= 6 && s[0] == '\\' && s[1] == 'u') {
            const unsigned lo = hex4(s + 2);
            if (lo < 0xDC00 || lo >= 0xE000) fail("bad surrogate pair");
            s += 6;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          if (cp < 0x80) {
            out.push_back(static_cast<char>(cp));
          } else if (cp < 0x800) {
            out.push_back(static_cast<char>(0xC0 | (cp >> 6)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
          } else if (cp < 0x10000) {
            out.push_back(static_cast<char>(0xE0 | (cp >> 12)));
            out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
          } else {
            out.push_back(static_cast<char>(0xF0 | (cp >> 18)));
            out.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back(static_cast<char>(0x80 | (cp & 0x3F)));
          }
          break;
        }
        default: fail("bad escape");
      }
    }
    if (s >= end) fail("unterminated string");
    ++s;
    return out;
  }

  // a JSON integer, parsed inside [s, end) only (never past the header) and overflow-checked
  int64_t integer() {
    ws();
    bool neg = false;
    if (s < end && (*s == '-' || *s == '+')) neg = *s++ == '-';
    if (s >= end || *s < '0' || *s > '9') fail("expected an integer");
    uint64_t v = 0;
    while (s < end && *s >= '0' && *s <= '9') {
      const unsigned d = static_cast<unsigned>(*s++ - '0');
      if (v > (static_cast<uint64_t>(INT64_MAX) - d) / 10) fail("integer out of range");
      v = v * 10 + d;
    }
    return neg ? -static_cast<int64_t>(v) : static_cast<int64_t>(v);
  }

  // the literal `w` at s (bounded by end); consumes it when present
  bool lit(const char* w) {
    const size_t k = std::strlen(w);
    if (static_cast<size_t>(end - s) < k || std::memcmp(s, w, k) != 0) return false;
    s += k;
    return true;
  }

  // a tensor descriptor must describe exactly its bytes: non-negative dims, nbytes = prod(shape) * element size
  // (overflow-checked), and [off, off + nbytes) inside the body
  void check_tensor(at::ScalarType dt, const std::vector<int64_t>& shape, int64_t off, int64_t nbytes) const {
    if (nbytes < 0 || off < 0) fail("negative tensor offset / size");
    uint64_t want = static_cast<uint64_t>(at::elementSize(dt));
    for (int64_t d : shape) {
      if (d < 0) fail("negative tensor dimension");
      if (d && want > static_cast<uint64_t>(INT64_MAX) / static_cast<uint64_t>(d)) fail("tensor size overflows");
      want *= static_cast<uint64_t>(d);
    }
    if (want != static_cast<uint64_t>(nbytes)) fail("tensor size mismatch");
    if (nbytes > body_len || off > body_len - nbytes) fail("tensor outside the body");
  }

  py::object value() {   // JSON scalar -> Python object
    ws();
    if (s >= end) fail("truncated header");
    if (*s == '"') return py::str(str());
    if (lit("null")) return py::none();
    if (lit("true")) return py::bool_(true);
    if (lit("false")) return py::bool_(false);
    if (lit("NaN")) return py::float_(std::nan(""));
    if (lit("Infinity")) return py::float_(INFINITY);
    if (lit("-Infinity")) return py::float_(-INFINITY);
    const char* st = s;
    bool is_float = false;
    if (s < end && (*s == '-' || *s == '+')) ++s;
    while (s < end && ((*s >= '0' && *s <= '9') || *s == '.' || *s == 'e' || *s == 'E' || *s == '-' || *s == '+')) {
      if (*s == '.' || *s == 'e' || *s == 'E') is_float = true;
      ++s;
    }
    std::string num(st, s);
    if (num.empty()) fail("bad value");
    if (is_float) {
      char* e = nullptr;
      const double v = std::strtod(num.c_str(), &e);
      if (e != num.c_str() + num.size()) fail("bad number");
      return py::float_(v);
    }
    // arbitrary-size ints through Python
    PyObject* v = PyLong_FromString(num.c_str(), nullptr, 10);
    if (!v) {
      PyErr_Clear();
      fail("bad integer");
    }
    return py::reinterpret_steal<py::object>(v);
  }

  py::object tensor_node() {   // after "__t__":
    expect('[');
    at::ScalarType dt;
    if (!dtype_from_code(str(), &dt)) fail("unknown dtype");
    expect(',');
    expect('[');
    std::vector<int64_t> shape;
    if (!peek(']')) {
      shape.push_back(integer());
      while (peek(',')) {
        ++s;
        shape.push_back(integer());
      }
    }
    expect(']');
    expect(',');
    const int64_t off = integer();
    expect(',');
    const int64_t nbytes = integer();
    expect(']');
    const auto opts = at::TensorOptions().dtype(dt);
    check_tensor(dt, shape, off, nbytes);
    if (nbytes == 0) return py::reinterpret_steal<py::object>(THPVariable_Wrap(at::empty(shape, opts)));
    at::Tensor t;
    if (copy) {
      t = at::empty(shape, opts);
      if (t.numel() * static_cast<int64_t>(t.element_size()) != nbytes) fail("tensor size mismatch");
      std::memcpy(t.data_ptr(), body + off, static_cast<size_t>(nbytes));
    } else {
      py::object keep = owner;
      auto* holder = new py::object(keep);
      t = at::from_blob(const_cast<uint8_t*>(body + off), shape, [holder](void*) {
            py::gil_scoped_acquire g;
            delete holder;
          }, opts);
      if (t.numel() * static_cast<int64_t>(t.element_size()) != nbytes) fail("tensor size mismatch");
    }
    return py::reinterpret_steal<py::object>(THPVariable_Wrap(t));
  }

  py::object node() {
    expect('{');
    const std::string tag = str();
    expect(':');
    py::object out;
    if (tag == "__t__") {
      out = tensor_node();
    } else if (tag == "__d__") {
      py::dict d;
      expect('[');
      bool first = true;
      while (!peek(']')) {
        if (!first) expect(',');
        first = false;
        expect('[');
        py::object k = peek('"') ? py::object(py::str(str())) : value();
        expect(',');
        d[k] = node();
        expect(']');
      }
      expect(']');
      out = d;
    } else if (tag == "__l__" || tag == "__tu__") {
      py::list l;
      expect('[');
      bool first = true;
      while (!peek(']')) {
        if (!first) expect(',');
        first = false;
        l.append(node());
      }
      expect(']');
      out = tag == "__l__" ? py::object(l) : py::object(py::tuple(l));
    } else if (tag == "__v__") {
      out = value();
    } else {
      fail("unknown node tag");
    }
    expect('}');
    return out;
  }
};

py::bytes frame_of(Encoder& enc);

py::bytes tree_dumps(py::handle tree) {
  Encoder enc;
  enc.header.reserve(8192);
  enc.node(tree);
  return frame_of(enc);
}

// one reply frame per batch row: row i of every batched tensor leaf (0-d leaves and non-tensor leaves as they
// are), leaf paths in `trims` narrowed to per-row lengths - the inference server's decollate + encode in one pass
std::vector<py::bytes> rows_dumps(py::handle tree, int64_t n, const Trims& trims) {
  std::vector<py::bytes> out;
  out.reserve(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    Encoder enc;
    enc.header.reserve(4096);
    enc.row = i;
    enc.trims = &trims;
    enc.node(tree);
    out.push_back(frame_of(enc));
  }
  return out;
}

py::bytes frame_of(Encoder& enc) {
  const int64_t hlen = static_cast<int64_t>(enc.header.size());
  const int64_t pre = static_cast<int64_t>(kMagicLen) + 9;
  const int64_t pad = (kAlign - (pre + hlen) % kAlign) % kAlign;
  const int64_t total = pre + hlen + pad + enc.offset;
  PyObject* out = PyBytes_FromStringAndSize(nullptr, static_cast<Py_ssize_t>(total));
  if (!out) throw py::error_already_set();
  char* dst = PyBytes_AS_STRING(out);
  std::memcpy(dst, kMagic, kMagicLen);
  const uint64_t hl = static_cast<uint64_t>(hlen);
  std::memcpy(dst + kMagicLen, &hl, 8);   // little endian (x86 / the '<Q' of the Python codec)
  dst[kMagicLen + 8] = 0;
  std::memcpy(dst + pre, enc.header.data(), static_cast<size_t>(hlen));
  char* body = dst + pre + hlen + pad;
  std::memset(dst + pre + hlen, 0, static_cast<size_t>(pad));
  {
    py::gil_scoped_release nogil;   // the copies touch no Python object
    int64_t cur = 0;
    for (const auto& b : enc.blobs) {
      if (b.first > cur) std::memset(body + cur, 0, static_cast<size_t>(b.first - cur));
      const int64_t n = b.second.numel() * static_cast<int64_t>(b.second.element_size());
      if (n) std::memcpy(body + b.first, b.second.data_ptr(), static_cast<size_t>(n));
      cur = b.first + n;
    }
  }
  return py::reinterpret_steal<py::bytes>(out);
}

py::object tree_loads(py::object data, bool copy) {
  py::buffer buf = py::reinterpret_borrow<py::buffer>(data);
  py::buffer_info info = buf.request();
  const auto* p = static_cast<const uint8_t*>(info.ptr);
  const int64_t n = static_cast<int64_t>(info.size * info.itemsize);
  const int64_t pre = static_cast<int64_t>(kMagicLen) + 9;
  if (n < pre || std::memcmp(p, kMagic, kMagicLen) != 0) throw py::value_error("not an applestar frame");
  uint64_t hlen = 0;
  std::memcpy(&hlen, p + kMagicLen, 8);
  if (p[kMagicLen + 8] != 0) throw py::value_error("tree_loads: compressed frame (use the Python codec)");
  if (hlen > static_cast<uint64_t>(n - pre)) throw py::value_error("tree_loads: truncated frame");
  const int64_t pad = (kAlign - (pre + static_cast<int64_t>(hlen)) % kAlign) % kAlign;
  const int64_t body_start = pre + static_cast<int64_t>(hlen) + pad;
  Decoder d;
  d.s = reinterpret_cast<const char*>(p + pre);
  d.end = d.s + hlen;
  d.body = p + body_start;
  d.body_len = n - body_start;
  d.copy = copy;
  d.owner = data;
  return d.node();
}

// ------------------------------------------------------------------------------------------------- trajectory index
// runtime/traj_ring.py: the learner's ingest thread needs, per trajectory frame, every step's tensor leaves (path,
// dtype, shape, body offset, bytes).  As json.loads + a Python tree walk that is ~20 ms per 64-step trajectory of
// GIL-held work (json.loads is one C call the interpreter cannot preempt) - at ~20 trajectories/s it starved the
// learner's launch thread (profiles/r5x_pipeline_*: 280 ms steps with ingest running, 45 ms without).  Here the
// header is parsed with the GIL released into one int64 table.
struct IdxKey {
  bool is_int = false;
  std::string s;
  int64_t i = 0;
  bool operator==(const IdxKey& o) const { return is_int == o.is_int && i == o.i && s == o.s; }
};
struct IdxLeaf {
  std::vector<IdxKey> path;
  std::string dt;
  std::vector<int64_t> shape;
  int64_t off = 0, nbytes = 0;
};

struct IndexParser : Decoder {
  std::vector<IdxKey> path;
  std::vector<IdxLeaf>* out = nullptr;

  void skip_value() {   // a JSON scalar (a __v__ payload): consumed, not built
    ws();
    if (s >= end) fail("truncated header");
    if (*s == '"') {
      str();
      return;
    }
    if (lit("null") || lit("true") || lit("false") || lit("NaN") || lit("Infinity") || lit("-Infinity")) return;
    const char* st = s;
    if (s < end && (*s == '-' || *s == '+')) ++s;
    while (s < end && ((*s >= '0' && *s <= '9') || *s == '.' || *s == 'e' || *s == 'E' || *s == '-' || *s == '+')) ++s;
    if (s == st) fail("bad value");
  }

  IdxKey key() {
    IdxKey k;
    if (peek('"')) {
      k.s = str();
    } else {
      k.is_int = true;
      k.i = integer();
    }
    return k;
  }

  void node() {
    expect('{');
    const std::string tag = str();
    expect(':');
    if (tag == "__t__") {
      IdxLeaf L;
      L.path = path;
      expect('[');
      L.dt = str();
      at::ScalarType dt;
      if (!dtype_from_code(L.dt, &dt)) fail("unknown dtype");
      expect(',');
      expect('[');
      if (!peek(']')) {
        L.shape.push_back(integer());
        while (peek(',')) {
          ++s;
          L.shape.push_back(integer());
        }
      }
      expect(']');
      expect(',');
      L.off = integer();
      expect(',');
      L.nbytes = integer();
      expect(']');
      check_tensor(dt, L.shape, L.off, L.nbytes);
      out->push_back(std::move(L));
    } else if (tag == "__d__") {
      expect('[');
      bool first = true;
      while (!peek(']')) {
        if (!first) expect(',');
        first = false;
        expect('[');
        path.push_back(key());
        expect(',');
        node();
        path.pop_back();
        expect(']');
      }
      expect(']');
    } else if (tag == "__l__" || tag == "__tu__") {
      expect('[');
      bool first = true;
      int64_t i = 0;
      while (!peek(']')) {
        if (!first) expect(',');
        first = false;
        IdxKey k;
        k.is_int = true;
        k.i = i++;
        path.push_back(k);
        node();
        path.pop_back();
      }
      expect(']');
    } else if (tag == "__v__") {
      skip_value();
    } else {
      fail("unknown node tag");
    }
    expect('}');
  }
};

constexpr int kIdxMaxDims = 4;

// frame -> (paths, dtype codes, meta int64 [T1, L, 3 + kIdxMaxDims] = body offset, nbytes (-1: absent in that
//           step), ndim, dims..., body offset of the frame) over the union of the steps' leaves; None when a path
//           changes dtype or a leaf has more than kIdxMaxDims dims (callers fall back)
py::object traj_index(py::object data) {
  py::buffer buf = py::reinterpret_borrow<py::buffer>(data);
  py::buffer_info info = buf.request();
  const auto* p = static_cast<const uint8_t*>(info.ptr);
  const int64_t n = static_cast<int64_t>(info.size * info.itemsize);
  const int64_t pre = static_cast<int64_t>(kMagicLen) + 9;
  if (n < pre || std::memcmp(p, kMagic, kMagicLen) != 0) throw py::value_error("not an applestar frame");
  uint64_t hlen = 0;
  std::memcpy(&hlen, p + kMagicLen, 8);
  if (p[kMagicLen + 8] != 0) throw py::value_error("traj_index: compressed frame");
  if (hlen > static_cast<uint64_t>(n - pre)) throw py::value_error("traj_index: truncated frame");
  const int64_t pad = (kAlign - (pre + static_cast<int64_t>(hlen)) % kAlign) % kAlign;
  const int64_t body_start = pre + static_cast<int64_t>(hlen) + pad;
  if (body_start > n) throw py::value_error("traj_index: truncated frame");
  std::vector<std::vector<IdxLeaf>> steps;
  std::map<std::string, int64_t> slot;
  std::vector<const IdxLeaf*> uni;
  bool layout_ok = true;
  {
    py::gil_scoped_release nogil;
    IndexParser d;
    d.s = reinterpret_cast<const char*>(p + pre);
    d.end = d.s + hlen;
    d.body = p + body_start;
    d.body_len = n - body_start;
    d.copy = false;
    d.expect('{');
    if (d.str() != "__l__") d.fail("traj_index: the header is not a step list");
    d.expect(':');
    d.expect('[');
    bool first = true;
    while (!d.peek(']')) {
      if (!first) d.expect(',');
      first = false;
      steps.emplace_back();
      d.out = &steps.back();
      d.node();
    }
    d.expect(']');
    d.expect('}');
    // the union of the steps' leaves in first-seen order (the last step carries only the observation, the first
    // the recurrent state); a path must keep its dtype
    for (const auto& st : steps)
      for (const IdxLeaf& lf : st) {
        if (lf.shape.size() > static_cast<size_t>(kIdxMaxDims)) layout_ok = false;
        std::string k;
        for (const IdxKey& q : lf.path) k += (q.is_int ? "i" + std::to_string(q.i) : "s" + q.s) + '\x1f';
        auto it = slot.find(k);
        if (it == slot.end()) {
          slot.emplace(k, static_cast<int64_t>(uni.size()));
          uni.push_back(&lf);
        } else if (uni[it->second]->dt != lf.dt) {
          layout_ok = false;
        }
      }
  }
  if (!layout_ok || steps.empty()) return py::none();
  const int64_t T1 = static_cast<int64_t>(steps.size()), L = static_cast<int64_t>(uni.size()),
                W = 3 + kIdxMaxDims;
  py::array_t<int64_t> meta({T1, L, W});
  auto* m = meta.mutable_data();
  for (int64_t i = 0; i < T1 * L; ++i) {
    int64_t* r = m + i * W;
    r[0] = 0;
    r[1] = -1;      // absent in this step
    r[2] = 0;
    for (int k = 0; k < kIdxMaxDims; ++k) r[3 + k] = 1;
  }
  for (int64_t t = 0; t < T1; ++t)
    for (const IdxLeaf& lf : steps[t]) {
      std::string k;
      for (const IdxKey& q : lf.path) k += (q.is_int ? "i" + std::to_string(q.i) : "s" + q.s) + '\x1f';
      int64_t* r = m + (t * L + slot[k]) * W;
      r[0] = lf.off;
      r[1] = lf.nbytes;
      r[2] = static_cast<int64_t>(lf.shape.size());
      for (size_t q = 0; q < lf.shape.size(); ++q) r[3 + q] = lf.shape[q];
    }
  py::list paths, dts;
  for (const IdxLeaf* lfp : uni) {
    const IdxLeaf& lf = *lfp;
    py::tuple tp(lf.path.size());
    for (size_t k = 0; k < lf.path.size(); ++k)
      tp[k] = lf.path[k].is_int ? py::object(py::int_(lf.path[k].i)) : py::object(py::str(lf.path[k].s));
    paths.append(tp);
    dts.append(py::str(lf.dt));
  }
  return py::make_tuple(paths, dts, meta, body_start);
}

// ------------------------------------------------------------------------------------------------- batch collate
// The inference server's per-batch host path: B request frames -> one pinned staging buffer laid out as the
// collated batch (agent/collate.py collate_obs: every leaf stacked on a new dim 0; entity_info leaves padded on
// their last dim to the batch's entity bucket; action_info/selected_units padded to 64) -> one H2D copy ->
// device views.  Replaces B frame decodes + ~110 torch.stack / pad calls + the pack-into-pinned copy.
struct Node {
  enum Kind { DICT, LIST, TUPLE, TENSOR, VALUE } kind = VALUE;
  std::vector<py::object> keys;
  std::vector<Node> kids;
  at::ScalarType dt = at::kByte;
  std::vector<int64_t> shape;
  int64_t off = 0, nbytes = 0;
  py::object value;
};

struct StructParser : Decoder {
  Node parse() {
    Node n;
    expect('{');
    const std::string tag = str();
    expect(':');
    if (tag == "__t__") {
      n.kind = Node::TENSOR;
      expect('[');
      if (!dtype_from_code(str(), &n.dt)) fail("unknown dtype");
      expect(',');
      expect('[');
      if (!peek(']')) {
        n.shape.push_back(integer());
        while (peek(',')) {
          ++s;
          n.shape.push_back(integer());
        }
      }
      expect(']');
      expect(',');
      n.off = integer();
      expect(',');
      n.nbytes = integer();
      expect(']');
      check_tensor(n.dt, n.shape, n.off, n.nbytes);
    } else if (tag == "__d__") {
      n.kind = Node::DICT;
      expect('[');
      bool first = true;
      while (!peek(']')) {
        if (!first) expect(',');
        first = false;
        expect('[');
        n.keys.push_back(peek('"') ? py::object(py::str(str())) : value());
        expect(',');
        n.kids.push_back(parse());
        expect(']');
      }
      expect(']');
    } else if (tag == "__l__" || tag == "__tu__") {
      n.kind = tag == "__l__" ? Node::LIST : Node::TUPLE;
      expect('[');
      bool first = true;
      while (!peek(']')) {
        if (!first) expect(',');
        first = false;
        n.kids.push_back(parse());
      }
      expect(']');
    } else if (tag == "__v__") {
      n.kind = Node::VALUE;
      n.value = value();
    } else {
      fail("unknown node tag");
    }
    expect('}');
    return n;
  }
};

struct Leaf {            // one collated tensor: B source slices -> one slot of the staging buffer
  at::ScalarType dt;
  std::vector<int64_t> shape;      // [B, ...] output shape
  int64_t off = 0;                 // byte offset in the staging buffer
  std::vector<const uint8_t*> src; // per-sample source bytes
  std::vector<int64_t> src_last;   // per-sample size of the (padded) last dim; -1: no padding
};

struct Collator {
  int64_t B = 0, pad_entities = 0, su_len = 64;
  std::vector<int64_t> buckets;    // entity-count buckets (ascending): the padded size is the first >= the max
  std::vector<const uint8_t*> bodies;
  std::vector<Leaf> leaves;
  int64_t total = 0;

  // returns the output-tree template: TENSOR nodes carry the leaf index in `off`
  Node plan(const std::vector<const Node*>& ns, const std::string& path, bool entity) {
    const Node& n0 = *ns[0];
    for (const Node* n : ns)
      if (n->kind != n0.kind || n->kids.size() != n0.kids.size())
        throw py::value_error("collate_frames: requests differ in structure at '" + path + "'");
    Node out;
    out.kind = n0.kind;
    if (n0.kind == Node::DICT || n0.kind == Node::LIST || n0.kind == Node::TUPLE) {
      out.keys = n0.keys;
      for (size_t i = 0; i < n0.kids.size(); ++i) {
        std::vector<const Node*> kids;
        for (const Node* n : ns) kids.push_back(&n->kids[i]);
        std::string key = n0.kind == Node::DICT ? py::str(n0.keys[i]).cast<std::string>() : std::to_string(i);
        const bool ent = entity || (path.empty() && n0.kind == Node::DICT && key == "entity_info");
        out.kids.push_back(plan(kids, path.empty() ? key : path + "/" + key, ent));
      }
      return out;
    }
    if (n0.kind == Node::VALUE) {
      py::list vals;
      for (const Node* n : ns) vals.append(n->value);
      out.value = vals;
      return out;
    }
    Leaf L;
    L.dt = n0.dt;
    const size_t rank = n0.shape.size();
    const bool su = path == "action_info/selected_units";
    const bool pad_last = rank >= 1 && (entity || su);
    int64_t last = rank ? n0.shape[rank - 1] : 0;
    for (const Node* n : ns) {
      if (n->dt != n0.dt || n->shape.size() != rank) throw py::value_error("collate_frames: dtype / rank differ at " + path);
      for (size_t d = 0; d + (pad_last ? 1 : 0) < rank; ++d)
        if (n->shape[d] != n0.shape[d]) throw py::value_error("collate_frames: shapes differ at " + path);
      if (pad_last) last = std::max(last, n->shape[rank - 1]);
    }
    if (pad_last) {
      if (su) {
        last = std::max(last, su_len);
      } else {
        last = std::max(last, pad_entities);
        for (int64_t b : buckets)
          if (b >= last) {
            last = b;
            break;
          }
      }
    }
    L.shape.push_back(B);
    for (size_t d = 0; d < rank; ++d) L.shape.push_back(pad_last && d == rank - 1 ? last : n0.shape[d]);
    for (size_t b = 0; b < ns.size(); ++b) {
      L.src.push_back(bodies[b] + ns[b]->off);
      L.src_last.push_back(pad_last ? ns[b]->shape[rank - 1] : -1);
    }
    int64_t bytes = at::elementSize(L.dt);
    for (int64_t d : L.shape) bytes *= d;
    L.off = (total + kAlign - 1) / kAlign * kAlign;
    total = L.off + bytes;
    out.off = static_cast<int64_t>(leaves.size());
    leaves.push_back(std::move(L));
    return out;
  }

  void copy_into(uint8_t* dst) const {
    for (const Leaf& L : leaves) {
      const int64_t es = at::elementSize(L.dt);
      int64_t per = es;      // bytes per sample
      for (size_t d = 1; d < L.shape.size(); ++d) per *= L.shape[d];
      for (int64_t b = 0; b < B; ++b) {
        uint8_t* o = dst + L.off + b * per;
        if (L.src_last[b] < 0) {
          std::memcpy(o, L.src[b], static_cast<size_t>(per));
          continue;
        }
        const int64_t out_last = L.shape.back();
        const int64_t rows = out_last ? per / (out_last * es) : 0;
        const int64_t in_row = L.src_last[b] * es, out_row = out_last * es;
        for (int64_t r = 0; r < rows; ++r) {
          std::memcpy(o + r * out_row, L.src[b] + r * in_row, static_cast<size_t>(in_row));
          std::memset(o + r * out_row + in_row, 0, static_cast<size_t>(out_row - in_row));
        }
      }
    }
  }

  py::object build(const Node& t, const at::Tensor& buf) const {
    switch (t.kind) {
      case Node::DICT: {
        py::dict d;
        for (size_t i = 0; i < t.kids.size(); ++i) d[t.keys[i]] = build(t.kids[i], buf);
        return d;
      }
      case Node::LIST:
      case Node::TUPLE: {
        py::list l;
        for (const Node& k : t.kids) l.append(build(k, buf));
        return t.kind == Node::LIST ? py::object(l) : py::object(py::tuple(l));
      }
      case Node::VALUE: {
        py::list vals = t.value;
        bool numeric = true;
        for (auto v : vals)
          if (!(PyLong_Check(v.ptr()) || PyFloat_Check(v.ptr()))) numeric = false;
        if (numeric && py::len(vals)) {
          py::object torch = py::module_::import("torch");
          return torch.attr("tensor")(vals);
        }
        return vals;
      }
      case Node::TENSOR: {
        const Leaf& L = leaves[static_cast<size_t>(t.off)];
        int64_t bytes = at::elementSize(L.dt);
        for (int64_t d : L.shape) bytes *= d;
        at::Tensor v = buf.narrow(0, L.off, bytes).view(L.dt).view(L.shape);
        return py::reinterpret_steal<py::object>(THPVariable_Wrap(v));
      }
    }
    return py::none();
  }
};

// frames: list of uncompressed frames of the same structure.  device: None -> host tensors; else the batch is
// staged in pinned memory and copied with ONE non_blocking H2D on the current stream.
py::object collate_frames(py::list frames, int64_t pad_entities, py::object device, std::vector<int64_t> buckets) {
  const int64_t B = static_cast<int64_t>(py::len(frames));
  if (B == 0) throw py::value_error("collate_frames: no frames");
  std::vector<Node> roots;
  Collator c;
  c.B = B;
  c.pad_entities = pad_entities;
  c.buckets = buckets;
  std::sort(c.buckets.begin(), c.buckets.end());
  std::vector<py::buffer_info> infos;
  for (auto f : frames) {
    py::buffer buf = py::reinterpret_borrow<py::buffer>(f);
    infos.push_back(buf.request());
    const auto* p = static_cast<const uint8_t*>(infos.back().ptr);
    const int64_t n = static_cast<int64_t>(infos.back().size * infos.back().itemsize);
    const int64_t pre = static_cast<int64_t>(kMagicLen) + 9;
    if (n < pre || std::memcmp(p, kMagic, kMagicLen) != 0 || p[kMagicLen + 8] != 0)
      throw py::value_error("collate_frames: not an uncompressed applestar frame");
    uint64_t hlen = 0;
    std::memcpy(&hlen, p + kMagicLen, 8);
    if (hlen > static_cast<uint64_t>(n - pre)) throw py::value_error("collate_frames: truncated frame");
    const int64_t pad = (kAlign - (pre + static_cast<int64_t>(hlen)) % kAlign) % kAlign;
    if (pre + static_cast<int64_t>(hlen) + pad > n) throw py::value_error("collate_frames: truncated frame");
    StructParser sp;
    sp.s = reinterpret_cast<const char*>(p + pre);
    sp.end = sp.s + hlen;
    sp.body = p + pre + static_cast<int64_t>(hlen) + pad;
    sp.body_len = n - (pre + static_cast<int64_t>(hlen) + pad);
    sp.copy = true;
    roots.push_back(sp.parse());
    c.bodies.push_back(sp.body);
  }
  std::vector<const Node*> rs;
  for (const Node& r : roots) rs.push_back(&r);
  const Node tmpl = c.plan(rs, "", false);
  const bool to_dev = !device.is_none();
  auto opts = at::TensorOptions().dtype(at::kByte);
  if (to_dev) opts = opts.pinned_memory(true);
  at::Tensor host = at::empty({std::max<int64_t>(c.total, 1)}, opts);
  {
    py::gil_scoped_release nogil;
    c.copy_into(host.data_ptr<uint8_t>());
  }
  at::Tensor buf = host;
  if (to_dev) {
    const at::Device dev(py::str(device).cast<std::string>());
    buf = host.to(dev, /*non_blocking=*/true);
  }
  return c.build(tmpl, buf);
}

}  // namespace

void register_codec(py::module& m) {
  m.def("tree_dumps", &tree_dumps, "tensor tree -> applestar frame (uncompressed)");
  m.def("tree_loads", &tree_loads, py::arg("data"), py::arg("copy") = true,
        "applestar frame -> tensor tree (copy=False: tensors alias the buffer)");
  m.def("rows_dumps", &rows_dumps, py::arg("tree"), py::arg("n"), py::arg("trims"),
        "one frame per batch row (row i of every batched leaf, per-path per-row narrowing)");
  m.def("traj_index", &traj_index, py::arg("data"),
        "trajectory frame -> (leaf paths, dtype codes, int64 [steps, leaves, 7] offsets / sizes / shapes, body start)");
  m.def("collate_frames", &collate_frames, py::arg("frames"), py::arg("pad_entities") = 0,
        py::arg("device") = py::none(), py::arg("buckets") = std::vector<int64_t>{}, "B request frames -> collated batch (one pinned staging buffer, one H2D)");
}
