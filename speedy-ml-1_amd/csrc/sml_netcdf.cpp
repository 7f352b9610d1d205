// sml_netcdf.cpp -- NetCDF-3 classic reader/writer for the per-region reservoir
// weight files, so trained weights load unchanged (no netCDF library needed).
//
// Reference writer: write_trained_res (src/mod_reservoir.f90:1701-1736) through
// write_netcdf_2d_non_met_data / write_netcdf_1d_non_met_data_{int,real}
// (src/mod_io.f90:1247-1496): one file per region, created NF90_CLOBBER (CDF-1,
// big-endian), variables win(win_x=n, win_y=ninp) and wout(wout_x=136,
// wout_y=n+132) as NF90_REAL, rows/cols(k) as NF90_INT, vals(k), mean(36),
// std(36) as NF90_REAL; each with a "units" attribute.  Fortran dimension order
// is reversed on disk, so the C-order shape of win is [ninp][n] and its bytes are
// exactly Fortran's column-major win(n, ninp).
// Reference reader: read_trained_res (src/mod_io.f90:2911-2956).
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sml_internal.hpp"

using namespace sml;

namespace {

enum { NC_DIMENSION = 10, NC_VARIABLE = 11, NC_ATTRIBUTE = 12 };
enum { NC_BYTE = 1, NC_CHAR = 2, NC_SHORT = 3, NC_INT = 4, NC_FLOAT = 5, NC_DOUBLE = 6 };

int type_size(int t) {
    switch (t) {
        case NC_BYTE:
        case NC_CHAR:
            return 1;
        case NC_SHORT:
            return 2;
        case NC_INT:
        case NC_FLOAT:
            return 4;
        case NC_DOUBLE:
            return 8;
    }
    return 0;
}

struct Var {
    std::string name;
    std::vector<int> dimids;
    int type = 0;
    int64_t begin = 0;
};

struct Reader {
    const std::vector<unsigned char> &b;
    size_t p = 0;
    bool ok = true;
    explicit Reader(const std::vector<unsigned char> &buf) : b(buf) {}
    uint32_t u32() {
        if (p + 4 > b.size()) {
            ok = false;
            return 0;
        }
        uint32_t v = ((uint32_t)b[p] << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
        p += 4;
        return v;
    }
    uint64_t u64() {
        uint64_t hi = u32();
        return (hi << 32) | u32();
    }
    std::string name() {
        uint32_t n = u32();
        if (!ok || p + n > b.size()) {
            ok = false;
            return {};
        }
        std::string s((const char *)&b[p], n);
        p += (n + 3) & ~3u;
        return s;
    }
    void skip_attrs() {
        uint32_t tag = u32(), count = u32();
        if (tag == 0) return;
        if (tag != NC_ATTRIBUTE) {
            ok = false;
            return;
        }
        for (uint32_t a = 0; a < count && ok; ++a) {
            name();
            int t = (int)u32();
            uint32_t ne = u32();
            size_t bytes = (size_t)ne * type_size(t);
            p += (bytes + 3) & ~(size_t)3;
        }
    }
};

int read_file(const char *path, std::vector<unsigned char> &buf) {
    FILE *f = std::fopen(path, "rb");
    if (!f) return fail(SML_ERR_IO, "cannot open %s", path);
    std::fseek(f, 0, SEEK_END);
    long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    buf.resize(sz > 0 ? (size_t)sz : 0);
    size_t got = buf.empty() ? 0 : std::fread(buf.data(), 1, buf.size(), f);
    std::fclose(f);
    if (got != buf.size()) return fail(SML_ERR_IO, "short read on %s", path);
    return SML_OK;
}

template <typename T>
void be_copy(const unsigned char *src, T *dst, size_t count) {
    for (size_t i = 0; i < count; ++i) {
        unsigned char tmp[sizeof(T)];
        for (size_t j = 0; j < sizeof(T); ++j) tmp[j] = src[i * sizeof(T) + sizeof(T) - 1 - j];
        std::memcpy(&dst[i], tmp, sizeof(T));
    }
}

}  // namespace

extern "C" int sml_nc_read_region(const char *path, int64_t *dims, float *win, float *wout, int *rows, int *cols,
                                  float *vals, float *mean, float *std) {
    SML_REQUIRE(path && dims, "null path/dims");
    std::vector<unsigned char> buf;
    if (int rc = read_file(path, buf)) return rc;
    if (buf.size() < 8 || buf[0] != 'C' || buf[1] != 'D' || buf[2] != 'F' || (buf[3] != 1 && buf[3] != 2))
        return fail(SML_ERR_FORMAT, "%s: not a NetCDF-3 classic / 64-bit-offset file", path);
    const bool off64 = buf[3] == 2;
    Reader r(buf);
    r.p = 4;
    r.u32();  // numrecs
    std::vector<int64_t> dimlen;
    {
        uint32_t tag = r.u32(), count = r.u32();
        if (tag == NC_DIMENSION)
            for (uint32_t d = 0; d < count && r.ok; ++d) {
                r.name();
                dimlen.push_back(r.u32());
            }
        else if (tag != 0)
            r.ok = false;
    }
    r.skip_attrs();  // global attributes
    std::vector<Var> vars;
    {
        uint32_t tag = r.u32(), count = r.u32();
        if (tag == NC_VARIABLE)
            for (uint32_t v = 0; v < count && r.ok; ++v) {
                Var var;
                var.name = r.name();
                uint32_t nd = r.u32();
                for (uint32_t d = 0; d < nd && r.ok; ++d) var.dimids.push_back((int)r.u32());
                r.skip_attrs();
                var.type = (int)r.u32();
                r.u32();  // vsize
                var.begin = off64 ? (int64_t)r.u64() : (int64_t)r.u32();
                vars.push_back(var);
            }
        else if (tag != 0)
            r.ok = false;
    }
    if (!r.ok) return fail(SML_ERR_FORMAT, "%s: malformed header", path);
    auto find = [&](const char *nm) -> const Var * {
        for (const Var &v : vars)
            if (v.name == nm) return &v;
        return nullptr;
    };
    auto shape = [&](const Var *v, int64_t *s0, int64_t *s1) -> bool {
        for (int d : v->dimids)
            if (d < 0 || d >= (int)dimlen.size()) return false;
        if (v->dimids.size() == 1) {
            *s0 = 1;
            *s1 = dimlen[v->dimids[0]];
            return true;
        }
        if (v->dimids.size() == 2) {
            *s0 = dimlen[v->dimids[0]];
            *s1 = dimlen[v->dimids[1]];
            return true;
        }
        return false;
    };
    const char *names[] = {"win", "wout", "rows", "cols", "vals", "mean", "std"};
    const Var *vp[7];
    int64_t sh[7][2];
    for (int i = 0; i < 7; ++i) {
        vp[i] = find(names[i]);
        if (!vp[i]) return fail(SML_ERR_FORMAT, "%s: variable '%s' missing", path, names[i]);
        if (!shape(vp[i], &sh[i][0], &sh[i][1])) return fail(SML_ERR_FORMAT, "%s: bad shape of '%s'", path, names[i]);
        const int want = (i == 2 || i == 3) ? NC_INT : NC_FLOAT;
        if (vp[i]->type != want)
            return fail(SML_ERR_FORMAT, "%s: '%s' has type %d, expected %d", path, names[i], vp[i]->type, want);
        const int64_t bytes = sh[i][0] * sh[i][1] * 4;
        if (vp[i]->begin < 0 || vp[i]->begin + bytes > (int64_t)buf.size())
            return fail(SML_ERR_FORMAT, "%s: '%s' data out of file bounds", path, names[i]);
    }
    dims[0] = sh[0][1];  // n      (win_x)
    dims[1] = sh[0][0];  // ninp   (win_y)
    dims[2] = sh[1][1];  // nout   (wout_x)
    dims[3] = sh[1][0];  // ncs+n  (wout_y)
    dims[4] = sh[2][1];  // k
    dims[5] = sh[5][1];  // 36
    if (sh[3][1] != dims[4] || sh[4][1] != dims[4] || sh[6][1] != dims[5])
        return fail(SML_ERR_FORMAT, "%s: inconsistent rows/cols/vals or mean/std lengths", path);
    auto data = [&](int i) { return buf.data() + vp[i]->begin; };
    if (win) be_copy(data(0), win, (size_t)(sh[0][0] * sh[0][1]));
    if (wout) be_copy(data(1), wout, (size_t)(sh[1][0] * sh[1][1]));
    if (rows) be_copy(data(2), rows, (size_t)dims[4]);
    if (cols) be_copy(data(3), cols, (size_t)dims[4]);
    if (vals) be_copy(data(4), vals, (size_t)dims[4]);
    if (mean) be_copy(data(5), mean, (size_t)dims[5]);
    if (std) be_copy(data(6), std, (size_t)dims[5]);
    return SML_OK;
}

namespace {
struct Writer {
    std::vector<unsigned char> b;
    void u32(uint32_t v) {
        for (int s = 24; s >= 0; s -= 8) b.push_back((unsigned char)(v >> s));
    }
    void name(const std::string &s) {
        u32((uint32_t)s.size());
        b.insert(b.end(), s.begin(), s.end());
        while (b.size() % 4) b.push_back(0);
    }
};
}  // namespace

extern "C" int sml_nc_write_region(const char *path, int n, int ninp, int nout, int ncs_plus_n, int k,
                                   const float *win, const float *wout, const int *rows, const int *cols,
                                   const float *vals, const float *mean, const float *std) {
    SML_REQUIRE(path && win && wout && rows && cols && vals && mean && std, "null argument");
    SML_REQUIRE(n > 0 && ninp > 0 && nout > 0 && ncs_plus_n >= n && k >= 0, "bad sizes");
    // dimension / variable order follows write_trained_res (mod_reservoir.f90:1725-1734)
    struct D {
        const char *name;
        int len;
    } dimv[] = {{"win_x", n},  {"win_y", ninp}, {"wout_x", nout}, {"wout_y", ncs_plus_n}, {"rows_x", k},
                {"cols_x", k}, {"vals_x", k},   {"mean_x", 36},   {"std_x", 36}};
    struct V {
        const char *name;
        int d0, d1;  // C-order dims (d0 = -1 for 1-D)
        int type;
        const void *data;
        int64_t count;
    } varv[] = {{"win", 1, 0, NC_FLOAT, win, (int64_t)n * ninp},
                {"wout", 3, 2, NC_FLOAT, wout, (int64_t)nout * ncs_plus_n},
                {"rows", -1, 4, NC_INT, rows, k},
                {"cols", -1, 5, NC_INT, cols, k},
                {"vals", -1, 6, NC_FLOAT, vals, k},
                {"mean", -1, 7, NC_FLOAT, mean, 36},
                {"std", -1, 8, NC_FLOAT, std, 36}};
    auto header = [&](const std::vector<uint32_t> &begins) {
        Writer w;
        w.b = {'C', 'D', 'F', 1};
        w.u32(0);
        w.u32(NC_DIMENSION);
        w.u32(9);
        for (const D &d : dimv) {
            w.name(d.name);
            w.u32((uint32_t)d.len);
        }
        w.u32(0);
        w.u32(0);  // no global attributes
        w.u32(NC_VARIABLE);
        w.u32(7);
        for (int i = 0; i < 7; ++i) {
            const V &v = varv[i];
            w.name(v.name);
            if (v.d0 >= 0) {
                w.u32(2);
                w.u32((uint32_t)v.d0);
                w.u32((uint32_t)v.d1);
            } else {
                w.u32(1);
                w.u32((uint32_t)v.d1);
            }
            w.u32(NC_ATTRIBUTE);
            w.u32(1);
            w.name("units");
            w.u32(NC_CHAR);
            w.u32(8);
            const char *u = "unitless";
            w.b.insert(w.b.end(), u, u + 8);
            w.u32(v.type);
            w.u32((uint32_t)((v.count * 4 + 3) & ~3LL));
            w.u32(begins[i]);
        }
        return w.b;
    };
    std::vector<uint32_t> begins(7, 0);
    size_t hsize = header(begins).size();
    uint64_t off = hsize;
    for (int i = 0; i < 7; ++i) {
        begins[i] = (uint32_t)off;
        off += (uint64_t)varv[i].count * 4;
        off = (off + 3) & ~3ull;
    }
    SML_REQUIRE(off < 0xFFFFFFFFull, "file too large for CDF-1");
    std::vector<unsigned char> out = header(begins);
    out.resize(off, 0);
    for (int i = 0; i < 7; ++i) {
        const unsigned char *src = (const unsigned char *)varv[i].data;
        unsigned char *dst = out.data() + begins[i];
        for (int64_t e = 0; e < varv[i].count; ++e)
            for (int j = 0; j < 4; ++j) dst[e * 4 + j] = src[e * 4 + 3 - j];
    }
    FILE *f = std::fopen(path, "wb");
    if (!f) return fail(SML_ERR_IO, "cannot create %s", path);
    size_t put = std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    if (put != out.size()) return fail(SML_ERR_IO, "short write on %s", path);
    return SML_OK;
}
