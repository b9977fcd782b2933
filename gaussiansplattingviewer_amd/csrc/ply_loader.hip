// ply_loader.hip -- native reader of 3D Gaussian Splatting PLY files (host code; SURVEY.md
// §8(f) row 2).
//
// Replaces util_gau.load_ply (reference util_gau.py:63-125), which parses with plyfile and
// per-property numpy loops -- the viewer's load-time bottleneck at 6M Gaussians.  Same
// contract: one `vertex` element with x y z, f_dc_0..2, exactly 45 f_rest_* (SH degree 3, the
// assertion at util_gau.py:94), opacity, scale_*, rot_*; the other properties (normals, ...)
// are ignored.  Output is the reference's activated SoA float32 data:
//   xyz      = float32(x, y, z)                                           (:65-67, :114)
//   rot      = float32(r / ||r||), r, ||r|| in float64, ||r|| = sqrt(((r0²+r1²)+r2²)+r3²)
//                                                                          (:110-116)
//   scale    = float32(exp(float64(raw)))                                  (:104-108, :118)
//   opacity  = sigmoid 1 / (1 + exp(-o)) in the property's precision (float32 for float
//              properties), then float32                                   (:69, :120)
//   sh[P,48] = f_dc_0..2, then for coefficient j = 0..14 the channels
//              (f_rest_j, f_rest_{15+j}, f_rest_{30+j})                   (:86-100, :122)
//   bbox     = per-axis min / max of xyz; center = per-axis float32 sum in vertex order
//              divided by float32(P) (numpy's mean over axis 0)            (:80-85)
// Parsing: memory-mapped file; binary_little_endian, binary_big_endian or ascii; any PLY
// scalar type per property (converted like numpy's astype).  Binary vertex records are
// converted in parallel (std::thread, contiguous vertex ranges); with device output the
// converted rows go through pinned staging chunks and hipMemcpyAsync on the caller's stream.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "gsr.h"

#define GSR_TRY_PLY(expr)             \
    do {                              \
        const int rc_ = (expr);       \
        if (rc_ != GSR_OK) return rc_; \
    } while (0)

int gsr_set_error(int code, const std::string &msg);  // api.hip

namespace {

int ply_fail(int code, const std::string &msg) { return gsr_set_error(code, "PLY: " + msg); }

enum class PType { I8, U8, I16, U16, I32, U32, F32, F64 };

bool ptype_of(const std::string &t, PType &out, int &size) {
    struct E {
        const char *n;
        PType t;
        int s;
    };
    static const E tab[] = {{"char", PType::I8, 1},    {"int8", PType::I8, 1},
                            {"uchar", PType::U8, 1},   {"uint8", PType::U8, 1},
                            {"short", PType::I16, 2},  {"int16", PType::I16, 2},
                            {"ushort", PType::U16, 2}, {"uint16", PType::U16, 2},
                            {"int", PType::I32, 4},    {"int32", PType::I32, 4},
                            {"uint", PType::U32, 4},   {"uint32", PType::U32, 4},
                            {"float", PType::F32, 4},  {"float32", PType::F32, 4},
                            {"double", PType::F64, 8}, {"float64", PType::F64, 8}};
    for (const E &e : tab)
        if (t == e.n) {
            out = e.t;
            size = e.s;
            return true;
        }
    return false;
}

struct Prop {
    std::string name;
    PType type;
    int size;
    int offset;  // within the binary vertex record
};

struct Header {
    enum Format { ASCII, BLE, BBE } format = BLE;
    int64_t count = 0;
    std::vector<Prop> props;
    int stride = 0;
    size_t data_offset = 0;  // first byte of the vertex element
};

// Field indices into Header::props of everything the loader reads.
struct Layout {
    int xyz[3], dc[3], rest[45], opacity, scale[3], rot[4];
    int n_scale = 0, n_rot = 0;
};

// A value of a property as double (exact for every PLY scalar type).
inline double read_value(const unsigned char *p, PType t, bool swap) {
    unsigned char b[8];
    int n = 0;
    switch (t) {
        case PType::I8: case PType::U8: n = 1; break;
        case PType::I16: case PType::U16: n = 2; break;
        case PType::I32: case PType::U32: case PType::F32: n = 4; break;
        case PType::F64: n = 8; break;
    }
    for (int i = 0; i < n; ++i) b[i] = swap ? p[n - 1 - i] : p[i];
    switch (t) {
        case PType::I8: { int8_t v; std::memcpy(&v, b, 1); return v; }
        case PType::U8: { uint8_t v; std::memcpy(&v, b, 1); return v; }
        case PType::I16: { int16_t v; std::memcpy(&v, b, 2); return v; }
        case PType::U16: { uint16_t v; std::memcpy(&v, b, 2); return v; }
        case PType::I32: { int32_t v; std::memcpy(&v, b, 4); return v; }
        case PType::U32: { uint32_t v; std::memcpy(&v, b, 4); return v; }
        case PType::F32: { float v; std::memcpy(&v, b, 4); return v; }
        case PType::F64: { double v; std::memcpy(&v, b, 8); return v; }
    }
    return 0.0;
}

// The reference builds xyz / opacity from the property arrays as read (float32 for float
// properties) and the other fields in float64: value as float32 = numpy astype(float32).
inline float as_f32(double v) { return (float)v; }

struct Mapped {
    const unsigned char *p = nullptr;
    size_t size = 0;
    ~Mapped() {
        if (p) munmap(const_cast<unsigned char *>(p), size);
    }
};

int map_file(const char *path, Mapped &m) {
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return ply_fail(GSR_E_INVALID, std::string("cannot open ") + path);
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size <= 0) {
        close(fd);
        return ply_fail(GSR_E_INVALID, std::string("cannot stat / empty file ") + path);
    }
    void *p = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (p == MAP_FAILED) return ply_fail(GSR_E_INVALID, std::string("mmap failed: ") + path);
    m.p = static_cast<const unsigned char *>(p);
    m.size = (size_t)st.st_size;
    return GSR_OK;
}

int parse_header(const Mapped &m, Header &h) {
    const char *s = reinterpret_cast<const char *>(m.p);
    const size_t n = m.size;
    size_t pos = 0;
    auto next_line = [&](std::string &line) -> bool {
        if (pos >= n) return false;
        size_t e = pos;
        while (e < n && s[e] != '\n') ++e;
        line.assign(s + pos, e - pos);
        if (!line.empty() && line.back() == '\r') line.pop_back();
        pos = e < n ? e + 1 : n;
        return true;
    };
    std::string line;
    if (!next_line(line) || line != "ply") return ply_fail(GSR_E_INVALID, "not a PLY file");
    bool in_vertex = false, seen_vertex = false, have_format = false;
    int64_t skip_bytes_before = 0;  // fixed-size elements before the vertex element
    int64_t cur_count = 0;
    int64_t cur_stride = 0;
    bool cur_has_list = false;
    // Counts and strides come from an untrusted header: every product and sum is bounded by
    // the file size before it is formed (no wrap in the size_t / int64 arithmetic below).
    auto close_element = [&]() -> int {
        if (!in_vertex && cur_count > 0 && !seen_vertex) {
            if (cur_has_list) return ply_fail(GSR_E_INVALID, "list property before the vertex element");
            const int64_t room = (int64_t)n - skip_bytes_before;  // skip_bytes_before <= n
            if (cur_stride > 0 && cur_count > room / cur_stride)
                return ply_fail(GSR_E_INVALID, "PLY file shorter than its elements");
            skip_bytes_before += cur_count * cur_stride;
        }
        return GSR_OK;
    };
    while (true) {
        if (!next_line(line)) return ply_fail(GSR_E_INVALID, "PLY header without end_header");
        char word[64] = {0};
        if (std::sscanf(line.c_str(), "%63s", word) != 1) continue;
        const std::string w = word;
        if (w == "comment" || w == "obj_info") continue;
        if (w == "format") {
            char fmt[64] = {0};
            std::sscanf(line.c_str(), "%*s %63s", fmt);
            const std::string f = fmt;
            if (f == "ascii") h.format = Header::ASCII;
            else if (f == "binary_little_endian") h.format = Header::BLE;
            else if (f == "binary_big_endian") h.format = Header::BBE;
            else return ply_fail(GSR_E_INVALID, "unknown PLY format " + f);
            have_format = true;
        } else if (w == "element") {
            GSR_TRY_PLY(close_element());
            char name[128] = {0};
            long long cnt = -1;
            if (std::sscanf(line.c_str(), "%*s %127s %lld", name, &cnt) != 2 || cnt < 0)
                return ply_fail(GSR_E_INVALID, "bad element line: " + line);
            in_vertex = std::string(name) == "vertex";
            if (in_vertex) {
                if (seen_vertex) return ply_fail(GSR_E_INVALID, "two vertex elements");
                seen_vertex = true;
                h.count = cnt;
            }
            cur_count = cnt;
            cur_stride = 0;
            cur_has_list = false;
        } else if (w == "property") {
            char t[64] = {0}, name[128] = {0};
            if (std::sscanf(line.c_str(), "%*s %63s", t) != 1)
                return ply_fail(GSR_E_INVALID, "bad property line: " + line);
            if (std::string(t) == "list") {
                if (in_vertex) return ply_fail(GSR_E_INVALID, "list property in the vertex element");
                cur_has_list = true;
                continue;
            }
            if (std::sscanf(line.c_str(), "%*s %*s %127s", name) != 1)
                return ply_fail(GSR_E_INVALID, "bad property line: " + line);
            PType pt;
            int sz;
            if (!ptype_of(t, pt, sz)) return ply_fail(GSR_E_INVALID, std::string("unknown type ") + t);
            if (cur_stride > (int64_t)n) return ply_fail(GSR_E_INVALID, "PLY element wider than the file");
            if (in_vertex) h.props.push_back({name, pt, sz, (int)cur_stride});
            cur_stride += sz;
            if (in_vertex) h.stride = (int)cur_stride;
        } else if (w == "end_header") {
            break;
        } else {
            return ply_fail(GSR_E_INVALID, "unexpected PLY header line: " + line);
        }
    }
    if (!have_format) return ply_fail(GSR_E_INVALID, "PLY header without format");
    if (!seen_vertex) return ply_fail(GSR_E_INVALID, "PLY file without a vertex element");
    h.data_offset = pos + (h.format == Header::ASCII ? 0 : (size_t)skip_bytes_before);
    if (h.format == Header::ASCII && skip_bytes_before > 0)
        return ply_fail(GSR_E_INVALID, "ascii PLY with elements before the vertex element");
    // ascii: every value takes at least two bytes ("0 "; the file's last one may end at EOF)
    if (h.format == Header::ASCII && !h.props.empty() &&
        (uint64_t)h.count > (m.size - std::min(m.size, h.data_offset) + 1) / (2 * h.props.size()))
        return ply_fail(GSR_E_INVALID, "ascii PLY shorter than its vertex data");
    if (h.format != Header::ASCII &&
        (h.data_offset > m.size ||
         (h.stride > 0 && (uint64_t)h.count > (m.size - h.data_offset) / (size_t)h.stride)))
        return ply_fail(GSR_E_INVALID, "PLY file shorter than its vertex data");
    return GSR_OK;
}

int find_prop(const Header &h, const std::string &name) {
    for (size_t i = 0; i < h.props.size(); ++i)
        if (h.props[i].name == name) return (int)i;
    return -1;
}

// Properties whose name starts with `prefix`, sorted by their integer suffix (the reference
// sorts with key int(name.split('_')[-1])).
std::vector<int> prefixed(const Header &h, const std::string &prefix) {
    std::vector<std::pair<long, int>> v;
    for (size_t i = 0; i < h.props.size(); ++i) {
        const std::string &n = h.props[i].name;
        if (n.compare(0, prefix.size(), prefix) != 0) continue;
        const size_t us = n.rfind('_');
        const long k = us == std::string::npos ? 0 : std::strtol(n.c_str() + us + 1, nullptr, 10);
        v.push_back({k, (int)i});
    }
    std::stable_sort(v.begin(), v.end(),
                     [](const std::pair<long, int> &a, const std::pair<long, int> &b) {
                         return a.first < b.first;
                     });
    std::vector<int> out;
    for (auto &e : v) out.push_back(e.second);
    return out;
}

int make_layout(const Header &h, Layout &L) {
    const char *xyz[3] = {"x", "y", "z"};
    for (int i = 0; i < 3; ++i)
        if ((L.xyz[i] = find_prop(h, xyz[i])) < 0)
            return ply_fail(GSR_E_INVALID, std::string("PLY vertex has no property ") + xyz[i]);
    for (int i = 0; i < 3; ++i) {
        const std::string n = "f_dc_" + std::to_string(i);
        if ((L.dc[i] = find_prop(h, n)) < 0)
            return ply_fail(GSR_E_INVALID, "PLY vertex has no property " + n);
    }
    if ((L.opacity = find_prop(h, "opacity")) < 0)
        return ply_fail(GSR_E_INVALID, "PLY vertex has no property opacity");
    const std::vector<int> rest = prefixed(h, "f_rest_");
    if (rest.size() != 45)  // util_gau.py:94: assert len(extra_f_names) == 3*(3+1)**2 - 3
        return ply_fail(GSR_E_INVALID, "expected 45 f_rest_* properties (SH degree 3), found " +
                                           std::to_string(rest.size()));
    for (int i = 0; i < 45; ++i) L.rest[i] = rest[i];
    const std::vector<int> sc = prefixed(h, "scale_"), ro = prefixed(h, "rot");
    if (sc.size() != 3) return ply_fail(GSR_E_INVALID, "expected 3 scale_* properties");
    if (ro.size() != 4) return ply_fail(GSR_E_INVALID, "expected 4 rot* properties");
    for (int i = 0; i < 3; ++i) L.scale[i] = sc[i];
    for (int i = 0; i < 4; ++i) L.rot[i] = ro[i];
    L.n_scale = 3;
    L.n_rot = 4;
    return GSR_OK;
}

// One vertex, activated (util_gau.py:114-124).  v = raw property values as double.
struct Row {
    float xyz[3], rot[4], scale[3], opacity, sh[48];
};

inline void activate(const double *v, const Layout &L, bool opacity_f32, Row &r) {
    for (int i = 0; i < 3; ++i) r.xyz[i] = as_f32(v[L.xyz[i]]);
    // rotation: the float64 array of the raw values (np.zeros + column copies), divided by its
    // L2 norm: sqrt of the sequential float64 sum of squares (numpy reduce over 4 elements)
    double q[4], ss = 0.0;
    for (int i = 0; i < 4; ++i) q[i] = v[L.rot[i]];
    for (int i = 0; i < 4; ++i) ss += q[i] * q[i];
    const double nrm = std::sqrt(ss);
    for (int i = 0; i < 4; ++i) r.rot[i] = (float)(q[i] / nrm);
    for (int i = 0; i < 3; ++i) r.scale[i] = (float)std::exp(v[L.scale[i]]);
    // opacity keeps the property's dtype in the reference: float32 sigmoid for float
    // properties (the usual case), float64 otherwise, then float32
    if (opacity_f32) {
        const float o = as_f32(v[L.opacity]);
        r.opacity = 1.0f / (1.0f + std::exp(-o));
    } else {
        r.opacity = (float)(1.0 / (1.0 + std::exp(-v[L.opacity])));
    }
    for (int c = 0; c < 3; ++c) r.sh[c] = as_f32(v[L.dc[c]]);
    for (int j = 0; j < 15; ++j)
        for (int c = 0; c < 3; ++c) r.sh[3 + 3 * j + c] = as_f32(v[L.rest[c * 15 + j]]);
}

// Convert vertices [b, e) of a binary file into the SoA host arrays.  Only the 59 fields the
// loader uses are decoded; little-endian float32 fields (the 3DGS files) take a direct load.
// Vertices [b, e) -> output rows (i - base) of the five arrays.
void convert_binary(const unsigned char *data, const Header &h, const Layout &L, int64_t b,
                    int64_t e, int64_t base, float *xyz, float *rot, float *scale, float *opacity,
                    float *sh) {
    const bool swap = h.format == Header::BBE;
    // field slots in `v` (indexed like Header::props, so activate() can use L unchanged)
    std::vector<int> need;
    for (int i = 0; i < 3; ++i) need.push_back(L.xyz[i]);
    for (int i = 0; i < 3; ++i) need.push_back(L.dc[i]);
    for (int i = 0; i < 45; ++i) need.push_back(L.rest[i]);
    need.push_back(L.opacity);
    for (int i = 0; i < 3; ++i) need.push_back(L.scale[i]);
    for (int i = 0; i < 4; ++i) need.push_back(L.rot[i]);
    struct Src {
        int slot, offset;
        PType type;
        bool fast;
    };
    std::vector<Src> src;
    for (int k : need) {
        const Prop &p = h.props[k];
        src.push_back({k, p.offset, p.type, p.type == PType::F32 && !swap});
    }
    std::vector<double> v(h.props.size(), 0.0);
    const bool op32 = h.props[L.opacity].type == PType::F32;
    Row r;
    for (int64_t i = b; i < e; ++i) {
        const unsigned char *rec = data + (size_t)i * (size_t)h.stride;
        for (const Src &f : src) {
            if (f.fast) {
                float x;
                std::memcpy(&x, rec + f.offset, 4);
                v[f.slot] = x;
            } else {
                v[f.slot] = read_value(rec + f.offset, f.type, swap);
            }
        }
        activate(v.data(), L, op32, r);
        const int64_t o = i - base;
        std::memcpy(xyz + 3 * o, r.xyz, 12);
        std::memcpy(rot + 4 * o, r.rot, 16);
        std::memcpy(scale + 3 * o, r.scale, 12);
        opacity[o] = r.opacity;
        std::memcpy(sh + 48 * o, r.sh, 192);
    }
}

// Converts vertices [b, e) with up to 16 threads (contiguous sub-ranges).
void convert_binary_parallel(const unsigned char *data, const Header &h, const Layout &L,
                             int64_t b, int64_t e, int64_t base, float *xyz, float *rot,
                             float *scale, float *opacity, float *sh) {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int64_t n = e - b;
    const int64_t nt = std::min<int64_t>(std::min<unsigned>(hw, 16u), std::max<int64_t>(1, n / 65536));
    if (nt == 1) {
        convert_binary(data, h, L, b, e, base, xyz, rot, scale, opacity, sh);
        return;
    }
    std::vector<std::thread> th;
    for (int64_t t = 0; t < nt; ++t)
        th.emplace_back(convert_binary, data, std::cref(h), std::cref(L), b + n * t / nt,
                        b + n * (t + 1) / nt, base, xyz, rot, scale, opacity, sh);
    for (auto &t : th) t.join();
}

// Binary file, float positions, device output: convert chunks of vertices straight into one of
// two pinned staging slots (SoA within the slot) and DMA each slot to the five device arrays
// while the next chunk converts -- the conversion (multi-threaded) and the upload overlap, and
// no full-size host copy is made.  Positions are also kept on the host for the bbox / mean.
int load_binary_to_device(const Mapped &m, const Header &h, const Layout &L, int64_t P,
                          float *xyz, float *rot, float *scale, float *opacity, float *sh,
                          hipStream_t s, std::vector<float> &host_xyz) {
    constexpr int64_t kRows = 1 << 18;             // vertices per chunk (~59 MB of output)
    constexpr int64_t kFloats = 3 + 4 + 3 + 1 + 48;
    const int64_t rows = std::min<int64_t>(kRows, P);
    float *pin = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&pin), 2 * (size_t)rows * kFloats * sizeof(float)) !=
        hipSuccess) {
        (void)hipGetLastError();
        return ply_fail(GSR_E_NOMEM, "pinned staging allocation failed");
    }
    host_xyz.resize((size_t)P * 3);
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool ok = hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) == hipSuccess;
    bool used[2] = {false, false};
    int slot = 0;
    for (int64_t b = 0; ok && b < P; b += rows) {
        const int64_t e = std::min(P, b + rows), n = e - b;
        if (used[slot]) ok = hipEventSynchronize(ev[slot]) == hipSuccess;
        if (!ok) break;
        float *sx = pin + (size_t)slot * rows * kFloats;
        float *sr = sx + 3 * n, *ss = sr + 4 * n, *so = ss + 3 * n, *ssh = so + n;
        convert_binary_parallel(m.p + h.data_offset, h, L, b, e, b, sx, sr, ss, so, ssh);
        std::memcpy(host_xyz.data() + 3 * b, sx, (size_t)n * 12);
        const struct {
            float *dst;
            const float *src;
            int64_t k;
        } parts[] = {{xyz, sx, 3}, {rot, sr, 4}, {scale, ss, 3}, {opacity, so, 1}, {sh, ssh, 48}};
        for (const auto &pt : parts)
            ok = ok && hipMemcpyAsync(pt.dst + pt.k * b, pt.src, (size_t)(pt.k * n) * sizeof(float),
                                      hipMemcpyHostToDevice, s) == hipSuccess;
        ok = ok && hipEventRecord(ev[slot], s) == hipSuccess;
        used[slot] = true;
        slot ^= 1;
    }
    ok = ok && hipStreamSynchronize(s) == hipSuccess;
    for (hipEvent_t x : ev)
        if (x) (void)hipEventDestroy(x);
    (void)hipHostFree(pin);
    if (!ok) {
        (void)hipGetLastError();
        return ply_fail(GSR_E_HIP, "upload of the PLY data failed");
    }
    return GSR_OK;
}

int convert_ascii(const Mapped &m, const Header &h, const Layout &L, float *xyz, float *rot,
                  float *scale, float *opacity, float *sh, double *xyz_raw) {
    const char *s = reinterpret_cast<const char *>(m.p) + h.data_offset;
    const char *end = reinterpret_cast<const char *>(m.p) + m.size;
    std::vector<double> v(h.props.size());
    Row r;
    for (int64_t i = 0; i < h.count; ++i) {
        for (size_t k = 0; k < h.props.size(); ++k) {
            while (s < end && (*s == ' ' || *s == '\n' || *s == '\r' || *s == '\t')) ++s;
            if (s >= end) return ply_fail(GSR_E_INVALID, "ascii PLY shorter than its vertex data");
            // the token, copied out NUL-terminated: strtod must not run past the mapping
            const char *t = s;
            while (t < end && !(*t == ' ' || *t == '\n' || *t == '\r' || *t == '\t')) ++t;
            char tok[64];
            const size_t len = (size_t)(t - s);
            if (len >= sizeof(tok)) return ply_fail(GSR_E_INVALID, "bad number in ascii PLY");
            std::memcpy(tok, s, len);
            tok[len] = '\0';
            char *stop = nullptr;
            // like plyfile (numpy text parsing): as float64, then the property's type
            const double d = std::strtod(tok, &stop);
            if (stop != tok + len || len == 0) return ply_fail(GSR_E_INVALID, "bad number in ascii PLY");
            s = t;
            double val = d;
            switch (h.props[k].type) {
                case PType::F32: val = (double)(float)d; break;
                case PType::F64: break;
                default: val = std::trunc(d); break;
            }
            v[k] = val;
        }
        activate(v.data(), L, h.props[L.opacity].type == PType::F32, r);
        std::memcpy(xyz + 3 * i, r.xyz, 12);
        std::memcpy(rot + 4 * i, r.rot, 16);
        std::memcpy(scale + 3 * i, r.scale, 12);
        opacity[i] = r.opacity;
        std::memcpy(sh + 48 * i, r.sh, 192);
        if (xyz_raw)  // double-typed positions: the reference's bbox / mean use these
            for (int c = 0; c < 3; ++c) xyz_raw[3 * i + c] = v[L.xyz[c]];
    }
    return GSR_OK;
}

// util_gau.py:80-85 on the positions as read (before the float32 cast): per-axis min / max
// (NaN propagates, as numpy's) and mean = sequential per-axis sum in vertex order / P, in the
// positions' own precision (T = float for float properties, double for double ones).
template <typename T>
void bbox_center(const T *xyz, int64_t P, float *mn, float *mx, float *center) {
    for (int c = 0; c < 3; ++c) {
        T lo = P ? xyz[c] : T(0), hi = lo, acc = T(0);
        for (int64_t i = 0; i < P; ++i) {
            const T x = xyz[3 * i + c];
            if (lo == lo && (x != x || x < lo)) lo = x;  // a NaN sticks, as in numpy
            if (hi == hi && (x != x || x > hi)) hi = x;
            acc += x;
        }
        mn[c] = (float)lo;
        mx[c] = (float)hi;
        center[c] = P ? (float)(acc / (T)P) : 0.0f;
    }
}

}  // namespace

extern "C" {

int gsr_ply_probe(const char *path, gsr_ply_info *info) {
    if (!path || !info) return ply_fail(GSR_E_INVALID, "gsr_ply_probe: NULL argument");
    std::memset(info, 0, sizeof(*info));
    Mapped m;
    GSR_TRY_PLY(map_file(path, m));
    Header h;
    GSR_TRY_PLY(parse_header(m, h));
    Layout L;
    GSR_TRY_PLY(make_layout(h, L));
    info->P = h.count;
    info->sh_coeffs = 16;
    info->binary = h.format != Header::ASCII;
    return GSR_OK;
}

int gsr_ply_load(const char *path, gsr_ply_info *info, float *xyz, float *rot, float *scale,
                 float *opacity, float *sh, int device, void *stream) {
    if (!path || !info || !xyz || !rot || !scale || !opacity || !sh)
        return ply_fail(GSR_E_INVALID, "gsr_ply_load: NULL argument");
    Mapped m;
    GSR_TRY_PLY(map_file(path, m));
    Header h;
    GSR_TRY_PLY(parse_header(m, h));
    Layout L;
    GSR_TRY_PLY(make_layout(h, L));
    if (info->P != 0 && info->P != h.count)
        return ply_fail(GSR_E_INVALID, "gsr_ply_load: info->P does not match the file (probe first)");
    const int64_t P = h.count;
    info->P = P;
    info->sh_coeffs = 16;
    info->binary = h.format != Header::ASCII;
    // positions of any non-float type: keep the raw values for the bbox / mean
    bool xyz_f32 = true;
    for (int c = 0; c < 3; ++c) xyz_f32 = xyz_f32 && h.props[L.xyz[c]].type == PType::F32;
    if (device && xyz_f32 && h.format != Header::ASCII && P > 0) {
        std::vector<float> host_xyz;
        GSR_TRY_PLY(load_binary_to_device(m, h, L, P, xyz, rot, scale, opacity, sh,
                                          static_cast<hipStream_t>(stream), host_xyz));
        bbox_center(host_xyz.data(), P, info->bbox_min, info->bbox_max, info->center);
        return GSR_OK;
    }
    // host staging: the caller's arrays, or a host copy that is uploaded afterwards (ascii
    // files and non-float positions)
    float *hx = xyz, *hr = rot, *hs = scale, *ho = opacity, *hsh = sh;
    std::vector<float> tmp;
    if (device) {
        tmp.resize((size_t)P * (3 + 4 + 3 + 1 + 48));
        hx = tmp.data();
        hr = hx + 3 * P;
        hs = hr + 4 * P;
        ho = hs + 3 * P;
        hsh = ho + P;
    }
    std::vector<double> xyz_raw(xyz_f32 ? 0 : (size_t)P * 3);
    if (h.format == Header::ASCII) {
        GSR_TRY_PLY(convert_ascii(m, h, L, hx, hr, hs, ho, hsh, xyz_f32 ? nullptr : xyz_raw.data()));
    } else {
        convert_binary_parallel(m.p + h.data_offset, h, L, 0, P, 0, hx, hr, hs, ho, hsh);
        if (!xyz_f32) {
            const bool swap = h.format == Header::BBE;
            for (int64_t i = 0; i < P; ++i)
                for (int c = 0; c < 3; ++c) {
                    const Prop &p = h.props[L.xyz[c]];
                    xyz_raw[3 * i + c] =
                        read_value(m.p + h.data_offset + (size_t)i * h.stride + p.offset, p.type, swap);
                }
        }
    }
    if (xyz_f32)
        bbox_center(hx, P, info->bbox_min, info->bbox_max, info->center);
    else
        bbox_center(xyz_raw.data(), P, info->bbox_min, info->bbox_max, info->center);
    if (device && P > 0) {
        hipStream_t s = static_cast<hipStream_t>(stream);
        struct Part {
            float *dst;
            const float *src;
            size_t n;
        } parts[] = {{xyz, hx, (size_t)P * 3}, {rot, hr, (size_t)P * 4}, {scale, hs, (size_t)P * 3},
                     {opacity, ho, (size_t)P}, {sh, hsh, (size_t)P * 48}};
        // pinned staging in 64 MiB chunks so the copies are asynchronous DMA
        const size_t chunk = (size_t)16 << 20;  // floats
        float *pin = nullptr;
        if (hipHostMalloc(reinterpret_cast<void **>(&pin), 2 * chunk * sizeof(float)) != hipSuccess) {
            (void)hipGetLastError();
            return ply_fail(GSR_E_NOMEM, "pinned staging allocation failed");
        }
        hipEvent_t ev[2] = {nullptr, nullptr};
        bool ok = hipEventCreateWithFlags(&ev[0], hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&ev[1], hipEventDisableTiming) == hipSuccess;
        int slot = 0;
        bool used[2] = {false, false};
        for (const Part &pt : parts) {
            for (size_t o = 0; ok && o < pt.n; o += chunk) {
                const size_t n = std::min(chunk, pt.n - o);
                if (used[slot]) ok = hipEventSynchronize(ev[slot]) == hipSuccess;
                float *buf = pin + slot * chunk;
                std::memcpy(buf, pt.src + o, n * sizeof(float));
                ok = ok && hipMemcpyAsync(pt.dst + o, buf, n * sizeof(float),
                                          hipMemcpyHostToDevice, s) == hipSuccess &&
                     hipEventRecord(ev[slot], s) == hipSuccess;
                used[slot] = true;
                slot ^= 1;
            }
        }
        ok = ok && hipStreamSynchronize(s) == hipSuccess;
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        (void)hipHostFree(pin);
        if (!ok) {
            (void)hipGetLastError();
            return ply_fail(GSR_E_HIP, "upload of the PLY data failed");
        }
    }
    return GSR_OK;
}

}  // extern "C"
