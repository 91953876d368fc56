/*
 * rt_ply.cpp — PLY mesh reader for raytrace_tris.
 *
 * Replaces the reference's PLYLoader (clrt/PLYLoader.cpp:4-90) over the vendored
 * ply.c reader (include/ply, read_ply / setup_property_ply / get_element_ply,
 * ply.c:2457-2720 for the binary/ascii element decoding).  Same semantics as the
 * reference's property table: vertex x, y, z read as float32 (PLYLoader.cpp:4-7,
 * any stored numeric type converted), face `vertex_indices` as a list of int32
 * with a uint8 count (PLYLoader.cpp:14-16; any integer count/item type accepted),
 * every other property and element skipped.  Differences, deliberate:
 *   - the reference copies a face only when vertCount == 2 (PLYLoader.cpp:74) and
 *     reads three indices of it — a bug that leaves every triangle uninitialised;
 *     here triangles are taken as stored and polygons are fan-triangulated
 *     (v0, v[k], v[k+1]); faces with < 3 vertices are dropped;
 *   - indices are range-checked (the reference would gather out of bounds).
 * Formats: ascii 1.0, binary_little_endian 1.0, binary_big_endian 1.0.
 * The whole body is decoded at open (one pass, streamed through a buffered
 * reader), so rt_ply_open reports exact vertex / triangle counts.
 */
#include <algorithm>
#include <cerrno>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "pathtracer_rt.h"
#include "rt_internal.h"

struct rt_ply {
    std::vector<float> verts;  /* xyz per vertex */
    std::vector<int32_t> tris; /* 3 indices per triangle */
    uint32_t dropped = 0;      /* faces with fewer than 3 vertices */
};

namespace {

enum Type { T_NONE, T_I8, T_U8, T_I16, T_U16, T_I32, T_U32, T_F32, T_F64 };

Type parse_type(const std::string &s)
{
    if (s == "char" || s == "int8") return T_I8;
    if (s == "uchar" || s == "uint8") return T_U8;
    if (s == "short" || s == "int16") return T_I16;
    if (s == "ushort" || s == "uint16") return T_U16;
    if (s == "int" || s == "int32") return T_I32;
    if (s == "uint" || s == "uint32") return T_U32;
    if (s == "float" || s == "float32") return T_F32;
    if (s == "double" || s == "float64") return T_F64;
    return T_NONE;
}

int type_size(Type t)
{
    switch (t) {
    case T_I8: case T_U8: return 1;
    case T_I16: case T_U16: return 2;
    case T_I32: case T_U32: case T_F32: return 4;
    case T_F64: return 8;
    default: return 0;
    }
}

struct Property {
    std::string name;
    Type type = T_NONE;       /* scalar type, or the item type of a list */
    Type count_type = T_NONE; /* != T_NONE: a list property */
};

struct Element {
    std::string name;
    uint64_t count = 0;
    std::vector<Property> props;
};

enum Format { F_ASCII, F_BLE, F_BBE };

/* Buffered byte / token reader over a FILE*. */
class Reader {
public:
    explicit Reader(FILE *f) : f_(f), buf_(1 << 20) {}
    bool get(void *dst, size_t n)
    {
        uint8_t *d = static_cast<uint8_t *>(dst);
        while (n) {
            if (pos_ == len_ && !fill()) return false;
            const size_t k = std::min(n, len_ - pos_);
            std::memcpy(d, buf_.data() + pos_, k);
            pos_ += k;
            d += k;
            n -= k;
        }
        return true;
    }
    int peek()
    {
        if (pos_ == len_ && !fill()) return EOF;
        return buf_[pos_];
    }
    int next()
    {
        const int c = peek();
        if (c != EOF) ++pos_;
        return c;
    }
    /* bytes of the file consumed so far */
    uint64_t consumed() const { return base_ + pos_; }
    /* one line without the newline; false at EOF with nothing read */
    bool line(std::string &s)
    {
        s.clear();
        int c;
        bool any = false;
        while ((c = next()) != EOF) {
            any = true;
            if (c == '\n') break;
            if (c != '\r') s.push_back((char)c);
        }
        return any;
    }
    /* next whitespace-separated token */
    bool token(std::string &s)
    {
        s.clear();
        int c;
        while ((c = peek()) != EOF && (c == ' ' || c == '\t' || c == '\n' || c == '\r')) ++pos_;
        while ((c = peek()) != EOF && !(c == ' ' || c == '\t' || c == '\n' || c == '\r')) {
            s.push_back((char)c);
            ++pos_;
        }
        return !s.empty();
    }

private:
    bool fill()
    {
        base_ += len_;
        len_ = std::fread(buf_.data(), 1, buf_.size(), f_);
        pos_ = 0;
        return len_ > 0;
    }
    FILE *f_;
    std::vector<uint8_t> buf_;
    size_t pos_ = 0, len_ = 0;
    uint64_t base_ = 0;
};

bool read_binary(Reader &r, Type t, bool big, double &v)
{
    uint8_t b[8];
    const int n = type_size(t);
    if (!r.get(b, (size_t)n)) return false;
    if (big) std::reverse(b, b + n);
    switch (t) {
    case T_I8: { int8_t x; std::memcpy(&x, b, 1); v = x; break; }
    case T_U8: v = b[0]; break;
    case T_I16: { int16_t x; std::memcpy(&x, b, 2); v = x; break; }
    case T_U16: { uint16_t x; std::memcpy(&x, b, 2); v = x; break; }
    case T_I32: { int32_t x; std::memcpy(&x, b, 4); v = x; break; }
    case T_U32: { uint32_t x; std::memcpy(&x, b, 4); v = x; break; }
    case T_F32: { float x; std::memcpy(&x, b, 4); v = x; break; }
    case T_F64: { double x; std::memcpy(&x, b, 8); v = x; break; }
    default: return false;
    }
    return true;
}

/* Scalars: x/y/z as float32 keep their exact bits (PLYLoader stores Float32). */
bool read_value(Reader &r, Format fmt, Type t, double &v, std::string &tok)
{
    if (fmt == F_ASCII) {
        if (!r.token(tok)) return false;
        char *end = nullptr;
        errno = 0;
        v = (t == T_F32 || t == T_F64) ? std::strtod(tok.c_str(), &end) : (double)std::strtoll(tok.c_str(), &end, 10);
        return end && *end == '\0' && errno == 0;
    }
    return read_binary(r, t, fmt == F_BBE, v);
}

std::string g_err;

/* The fewest bytes one stored value of type t can take: its size in a binary body; in an ascii
   body one character (the separator may be the end of the file) */
uint64_t min_value_bytes(Format fmt, Type t) { return fmt == F_ASCII ? 1u : (uint64_t)type_size(t); }

/* The fewest bytes one instance of element e can take (a list counts its count only) */
uint64_t min_element_bytes(Format fmt, const Element &e)
{
    uint64_t b = 0;
    for (const Property &p : e.props) b += min_value_bytes(fmt, p.count_type != T_NONE ? p.count_type : p.type);
    return b;
}

/* The body is checked against the header before anything is sized from it: an element count
   (or a list length) the rest of the file cannot hold is a malformed file, reported as such
   instead of a multi-gigabyte allocation (a header saying `element face 4000000000000000000`
   used to end in std::length_error). */
struct Malformed {
    const char *what;
};

} // namespace

extern "C" {

const char *rt_ply_last_error(void) { return g_err.c_str(); }

int rt_ply_open(const char *path, rt_ply **out, uint32_t *n_verts, uint32_t *n_tris)
try {
    g_err.clear();
    if (!path || !out) return RT_ERR_ARG;
    *out = nullptr;
    FILE *f = std::fopen(path, "rb");
    if (!f) {
        g_err = std::string("cannot open ") + path;
        return RT_ERR_ARG;
    }
    std::unique_ptr<FILE, int (*)(FILE *)> guard(f, std::fclose);
    Reader r(f);
    std::string ln;
    if (!r.line(ln) || ln != "ply") {
        g_err = "not a PLY file (missing 'ply' magic)";
        return RT_ERR_ARG;
    }
    Format fmt = F_ASCII;
    bool have_fmt = false;
    std::vector<Element> elems;
    for (;;) {
        if (!r.line(ln)) {
            g_err = "truncated header";
            return RT_ERR_ARG;
        }
        char w0[64] = {0}, w1[64] = {0}, w2[64] = {0}, w3[64] = {0}, w4[256] = {0};
        const int nw = std::sscanf(ln.c_str(), "%63s %63s %63s %63s %255s", w0, w1, w2, w3, w4);
        if (nw <= 0) continue;
        const std::string k = w0;
        if (k == "end_header") break;
        if (k == "comment" || k == "obj_info") continue;
        if (k == "format") {
            const std::string f1 = w1;
            if (f1 == "ascii") fmt = F_ASCII;
            else if (f1 == "binary_little_endian") fmt = F_BLE;
            else if (f1 == "binary_big_endian") fmt = F_BBE;
            else {
                g_err = "unknown PLY format " + f1;
                return RT_ERR_ARG;
            }
            have_fmt = true;
        } else if (k == "element") {
            if (nw < 3) {
                g_err = "bad element line";
                return RT_ERR_ARG;
            }
            Element e;
            e.name = w1;
            e.count = std::strtoull(w2, nullptr, 10);
            elems.push_back(e);
        } else if (k == "property") {
            if (elems.empty()) {
                g_err = "property before any element";
                return RT_ERR_ARG;
            }
            Property p;
            if (std::string(w1) == "list") {
                if (nw < 5) {
                    g_err = "bad list property";
                    return RT_ERR_ARG;
                }
                p.count_type = parse_type(w2);
                p.type = parse_type(w3);
                p.name = w4;
                if (p.count_type == T_NONE || p.type == T_NONE || p.count_type == T_F32 || p.count_type == T_F64) {
                    g_err = "bad list types";
                    return RT_ERR_ARG;
                }
            } else {
                p.type = parse_type(w1);
                p.name = w2;
                if (p.type == T_NONE) {
                    g_err = std::string("unknown property type ") + w1;
                    return RT_ERR_ARG;
                }
            }
            elems.back().props.push_back(p);
        } else {
            g_err = "unknown header line: " + ln;
            return RT_ERR_ARG;
        }
    }
    if (!have_fmt) {
        g_err = "missing format line";
        return RT_ERR_ARG;
    }
    uint64_t file_bytes = 0;
    {
        const long here = std::ftell(f);
        if (here < 0 || std::fseek(f, 0, SEEK_END) != 0) {
            g_err = "cannot size the file";
            return RT_ERR_ARG;
        }
        const long end = std::ftell(f);
        if (end < 0 || std::fseek(f, here, SEEK_SET) != 0) {
            g_err = "cannot size the file";
            return RT_ERR_ARG;
        }
        file_bytes = (uint64_t)end;
    }
    {
        uint64_t left = file_bytes > r.consumed() ? file_bytes - r.consumed() : 0;
        for (const Element &e : elems) {
            const uint64_t per = min_element_bytes(fmt, e);
            if (per && e.count > left / per) {
                g_err = "element " + e.name + " declares " + std::to_string(e.count) + " instances of at least " +
                        std::to_string(per) + " bytes, but the body has " + std::to_string(left) + " bytes left";
                return RT_ERR_ARG;
            }
            if (!per && e.count) { /* no properties: nothing to read, and nothing bounds the count */
                g_err = "element " + e.name + " has instances but no properties";
                return RT_ERR_ARG;
            }
            left -= per * e.count;
        }
    }
    std::unique_ptr<rt_ply> ply(new (std::nothrow) rt_ply);
    if (!ply) return RT_ERR_ALLOC;
    uint64_t nv_total = 0;
    bool have_vertex = false;
    std::string tok;
    try {
        for (const Element &e : elems) {
            const bool is_vertex = e.name == "vertex";
            const bool is_face = e.name == "face";
            int ix = -1, iy = -1, iz = -1, ilist = -1;
            for (size_t i = 0; i < e.props.size(); ++i) {
                const Property &p = e.props[i];
                if (is_vertex && p.count_type == T_NONE) {
                    if (p.name == "x") ix = (int)i;
                    if (p.name == "y") iy = (int)i;
                    if (p.name == "z") iz = (int)i;
                }
                if (is_face && p.count_type != T_NONE && (p.name == "vertex_indices" || p.name == "vertex_index"))
                    ilist = (int)i;
            }
            if (is_vertex) {
                if (ix < 0 || iy < 0 || iz < 0) {
                    g_err = "vertex element without x, y, z";
                    return RT_ERR_ARG;
                }
                if (e.count > 0xFFFFFFFFull) {
                    g_err = "too many vertices";
                    return RT_ERR_LIMIT;
                }
                ply->verts.resize(3 * e.count);
                nv_total = e.count;
                have_vertex = true;
            }
            if (is_face && ilist < 0) {
                g_err = "face element without vertex_indices";
                return RT_ERR_ARG;
            }
            if (is_face) ply->tris.reserve((size_t)std::min<uint64_t>(3 * e.count, 1ull << 26)); /* fans may add more */
            std::vector<int64_t> face;
            for (uint64_t j = 0; j < e.count; ++j) {
                for (size_t i = 0; i < e.props.size(); ++i) {
                    const Property &p = e.props[i];
                    double v = 0;
                    if (p.count_type != T_NONE) {
                        double cnt = 0;
                        if (!read_value(r, fmt, p.count_type, cnt, tok)) throw 1;
                        if (!(cnt >= 0)) throw Malformed{"negative list length"};
                        const uint64_t n = (uint64_t)cnt; /* an integer type's value: exact, below 2^32 */
                        const uint64_t item = min_value_bytes(fmt, p.type);
                        const uint64_t left = file_bytes > r.consumed() ? file_bytes - r.consumed() : 0;
                        if (item && n > left / item) throw Malformed{"truncated (a list runs past the end of the file)"};
                        const bool keep = is_face && (int)i == ilist;
                        if (keep) face.clear();
                        for (uint64_t q = 0; q < n; ++q) {
                            if (!read_value(r, fmt, p.type, v, tok)) throw 1;
                            if (keep) {
                                if (!(v >= 0.0 && v < 2147483647.0)) throw Malformed{"face index out of range"};
                                face.push_back((int64_t)v);
                            }
                        }
                        continue;
                    }
                    if (!read_value(r, fmt, p.type, v, tok)) throw 1;
                    if (is_vertex && ((int)i == ix || (int)i == iy || (int)i == iz) && !(std::fabs(v) <= (double)FLT_MAX))
                        throw Malformed{"vertex coordinate not a finite float"};
                    if (is_vertex) {
                        if ((int)i == ix) ply->verts[3 * j + 0] = (float)v;
                        else if ((int)i == iy) ply->verts[3 * j + 1] = (float)v;
                        else if ((int)i == iz) ply->verts[3 * j + 2] = (float)v;
                    }
                }
                if (is_face) {
                    if (face.size() < 3) {
                        ply->dropped++;
                        continue;
                    }
                    for (size_t q = 1; q + 1 < face.size(); ++q) { /* fan: (v0, v[q], v[q+1]) */
                        ply->tris.push_back((int32_t)face[0]);
                        ply->tris.push_back((int32_t)face[q]);
                        ply->tris.push_back((int32_t)face[q + 1]);
                    }
                }
            }
        }
    } catch (int) {
        g_err = "truncated or malformed PLY body";
        return RT_ERR_ARG;
    } catch (const Malformed &m) {
        g_err = std::string("malformed PLY body: ") + m.what;
        return RT_ERR_ARG;
    } catch (const std::bad_alloc &) {
        g_err = "out of memory";
        return RT_ERR_ALLOC;
    }
    if (!have_vertex) {
        g_err = "no vertex element";
        return RT_ERR_ARG;
    }
    for (int32_t vi : ply->tris)
        if ((uint64_t)vi >= nv_total) {
            g_err = "face index out of range";
            return RT_ERR_ARG;
        }
    if (ply->tris.size() / 3 > 0xFFFFFFFFull) {
        g_err = "too many triangles";
        return RT_ERR_LIMIT;
    }
    if (n_verts) *n_verts = (uint32_t)nv_total;
    if (n_tris) *n_tris = (uint32_t)(ply->tris.size() / 3);
    *out = ply.release();
    return RT_OK;
} RT_CATCH(&g_err)

int rt_ply_read(const rt_ply *ply, float *verts_xyz, int32_t *idx)
try {
    if (!ply || (!verts_xyz && !ply->verts.empty()) || (!idx && !ply->tris.empty())) return RT_ERR_ARG;
    if (!ply->verts.empty()) std::memcpy(verts_xyz, ply->verts.data(), ply->verts.size() * sizeof(float));
    if (!ply->tris.empty()) std::memcpy(idx, ply->tris.data(), ply->tris.size() * sizeof(int32_t));
    return RT_OK;
} RT_CATCH(&g_err)

uint32_t rt_ply_dropped_faces(const rt_ply *ply) { return ply ? ply->dropped : 0u; }

int rt_ply_close(rt_ply *ply)
try {
    delete ply;
    return RT_OK;
} RT_CATCH(&g_err)

int rt_normalize_mesh(float *verts_xyz, uint32_t n_verts, float max_extent, float floor_y)
try {
    if (!verts_xyz || !n_verts || !(max_extent > 0)) return RT_ERR_ARG;
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = 0; i < n_verts; ++i)
        for (int a = 0; a < 3; ++a) {
            const double v = verts_xyz[3ull * i + a];
            if (!std::isfinite(v)) return RT_ERR_ARG;
            lo[a] = std::min(lo[a], v);
            hi[a] = std::max(hi[a], v);
        }
    const double ext = std::max(hi[0] - lo[0], std::max(hi[1] - lo[1], hi[2] - lo[2]));
    const double s = ext > 0 ? (double)max_extent / ext : 1.0;
    const double cx = 0.5 * (lo[0] + hi[0]), cz = 0.5 * (lo[2] + hi[2]);
    for (uint32_t i = 0; i < n_verts; ++i) {
        float *v = verts_xyz + 3ull * i;
        v[0] = (float)((v[0] - cx) * s);
        v[1] = (float)((v[1] - lo[1]) * s + floor_y);
        v[2] = (float)((v[2] - cz) * s);
    }
    return RT_OK;
} RT_CATCH(nullptr)

} /* extern "C" */
