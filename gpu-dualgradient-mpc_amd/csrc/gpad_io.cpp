// gpad_io.cpp -- the reference's text data-file boundary (main.cu:29-67 readData).
//
// Layout of the file (as readData consumes it, non-flattened build):
//   "n_u N m num_iterations L"  then  M_G[N*n_u*m]  g_P[N*n_u]  G_L[N*n_u*m]  p_D[m]
//   theta[num_iterations]  beta[num_iterations]
// Values are parsed as fscanf("%f") does (strtof).  Differences from readData, deliberate:
// a truncated or malformed file is an error (readData perror()s and continues with garbage),
// and the matrix layout is explicit (GPAD_FILE_ROWMAJOR / GPAD_FILE_FLIPPED, see gpad.h).
// The writer prints every float with 9 significant digits, so write -> read is exact.
#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gpad.h"
#include "gpad_abi.h"
#include "gpad_internal.h"

namespace {

int io_fail(const std::string& msg) { return gpad::set_last_error(GPAD_ERR_INVALID, msg); }

struct Reader {
    std::vector<char> buf;
    size_t pos = 0;
    bool next(const char** start) {
        while (pos < buf.size() && (buf[pos] == ' ' || buf[pos] == '\n' || buf[pos] == '\t' ||
                                    buf[pos] == '\r' || buf[pos] == '\v' || buf[pos] == '\f'))
            ++pos;
        if (pos >= buf.size() || buf[pos] == '\0') return false;
        *start = &buf[pos];
        return true;
    }
    bool read_int(int* out) {
        const char* s;
        if (!next(&s)) return false;
        char* end;
        errno = 0;
        long v = std::strtol(s, &end, 10);
        if (end == s || errno || v < INT_MIN || v > INT_MAX) return false;
        pos += (size_t)(end - s);
        *out = (int)v;
        return true;
    }
    bool read_float(float* out) {
        const char* s;
        if (!next(&s)) return false;
        char* end;
        float v = std::strtof(s, &end);
        if (end == s) return false;
        pos += (size_t)(end - s);
        *out = v;
        return true;
    }
    bool read_floats(float* out, size_t count) {
        for (size_t i = 0; i < count; ++i)
            if (!read_float(&out[i])) return false;
        return true;
    }
};

// row-major (rows x cols) <-> flipped storage (cols x rows)
void transpose(const float* in, float* out, int rows, int cols) {
    for (int i = 0; i < rows; ++i)
        for (int j = 0; j < cols; ++j) out[(size_t)i * cols + j] = in[(size_t)j * rows + i];
}

}  // namespace

extern "C" {

void gpad_datafile_free(gpad_datafile_t* f) {
    if (!f) return;
    std::free(f->M_G);
    std::free(f->g_P);
    std::free(f->G_L);
    std::free(f->p_D);
    std::free(f->theta);
    std::free(f->beta);
    f->M_G = f->g_P = f->G_L = f->p_D = f->theta = f->beta = nullptr;
}

int gpad_datafile_read(const char* path, int layout, gpad_datafile_t* out) {
    return gpad::abi_guard("gpad_datafile_read", [&]() -> int {
        if (!path || !out) return io_fail("gpad_datafile_read: null argument");
        if (layout != GPAD_FILE_ROWMAJOR && layout != GPAD_FILE_FLIPPED && layout != GPAD_FILE_FLAT)
            return io_fail("gpad_datafile_read: bad layout");
        std::memset(out, 0, sizeof(*out));
        FILE* fp = std::fopen(path, "rb");
        if (!fp) return io_fail(std::string("gpad_datafile_read: cannot open ") + path);
        Reader r;
        char chunk[1 << 16];
        size_t got;
        while ((got = std::fread(chunk, 1, sizeof(chunk), fp)) > 0) r.buf.insert(r.buf.end(), chunk, chunk + got);
        std::fclose(fp);
        r.buf.push_back('\0');
        gpad_datafile_t f{};
        if (!r.read_int(&f.n_u) || !r.read_int(&f.N) || !r.read_int(&f.m) || !r.read_int(&f.num_iterations) ||
            !r.read_float(&f.L))
            return io_fail("gpad_datafile_read: bad header (expected n_u N m num_iterations L)");
        if (f.n_u <= 0 || f.N <= 0 || f.m <= 0 || f.num_iterations < 0)
            return io_fail("gpad_datafile_read: header sizes must be positive");
        // The values the header announces must fit the file (each takes at least one character and a
        // separator), which also bounds every allocation below by the file's size -- a corrupted
        // header must not size a multi-GB buffer or overflow n = n_u N.
        const unsigned long long n64 = (unsigned long long)f.n_u * (unsigned long long)f.N;
        const unsigned long long rows64 = layout == GPAD_FILE_FLAT ? (unsigned long long)f.N : n64;
        const unsigned long long nm64 = rows64 * (unsigned long long)f.m;
        const unsigned long long values = 2 * nm64 + n64 + (unsigned long long)f.m + 2ull * (unsigned long long)f.num_iterations;
        if (n64 > (unsigned long long)INT_MAX || values > (r.buf.size() - r.pos + 1) / 2 + 1)
            return io_fail("gpad_datafile_read: header sizes exceed the data in " + std::string(path));
        const int n = (int)n64, m = f.m;
        // flat files hold N x m / m x N matrices (main.cu:39-56 under ENABLE_FLATTEN_MATRICES)
        const size_t nm = (size_t)nm64;
        auto alloc = [](size_t k) { return (float*)std::calloc(k ? k : 1, sizeof(float)); };
        f.M_G = alloc(nm);
        f.g_P = alloc(n);
        f.G_L = alloc(nm);
        f.p_D = alloc(m);
        f.theta = alloc(f.num_iterations);
        f.beta = alloc(f.num_iterations);
        std::vector<float> tmp(layout == GPAD_FILE_FLIPPED ? nm : 0);  // (the flipped layout's transpose)
        bool ok = f.M_G && f.g_P && f.G_L && f.p_D && f.theta && f.beta;
        if (ok) {
            // M_G: n x m row-major, or flipped [j*n + i] (an m x n array)
            ok = r.read_floats(layout == GPAD_FILE_FLIPPED ? tmp.data() : f.M_G, nm);
            if (ok && layout == GPAD_FILE_FLIPPED) transpose(tmp.data(), f.M_G, n, m);
            ok = ok && r.read_floats(f.g_P, n);
            // G_L: m x n row-major, or flipped [j*m + i] (an n x m array)
            ok = ok && r.read_floats(layout == GPAD_FILE_FLIPPED ? tmp.data() : f.G_L, nm);
            if (ok && layout == GPAD_FILE_FLIPPED) transpose(tmp.data(), f.G_L, m, n);
            ok = ok && r.read_floats(f.p_D, m) && r.read_floats(f.theta, f.num_iterations) &&
                 r.read_floats(f.beta, f.num_iterations);
        }
        if (!ok) {
            gpad_datafile_free(&f);
            return io_fail("gpad_datafile_read: truncated or malformed data in " + std::string(path));
        }
        *out = f;
        return GPAD_OK;
    });
}

int gpad_datafile_write(const char* path, int layout, const gpad_datafile_t* f) {
    return gpad::abi_guard("gpad_datafile_write", [&]() -> int {
        if (!path || !f || !f->M_G || !f->g_P || !f->G_L || !f->p_D ||
            (f->num_iterations > 0 && (!f->theta || !f->beta)))
            return io_fail("gpad_datafile_write: null argument");
        if (layout != GPAD_FILE_ROWMAJOR && layout != GPAD_FILE_FLIPPED && layout != GPAD_FILE_FLAT)
            return io_fail("gpad_datafile_write: bad layout");
        if (f->n_u <= 0 || f->N <= 0 || f->m <= 0 || f->num_iterations < 0)
            return io_fail("gpad_datafile_write: bad sizes");
        FILE* fp = std::fopen(path, "w");
        if (!fp) return io_fail(std::string("gpad_datafile_write: cannot open ") + path);
        const int n = f->n_u * f->N, m = f->m;
        std::fprintf(fp, "%d %d %d %d %.9g\n", f->n_u, f->N, f->m, f->num_iterations, (double)f->L);
        auto vec = [&](const float* v, size_t k) {
            for (size_t i = 0; i < k; ++i) std::fprintf(fp, i + 1 == k ? "%.9g\n" : "%.9g ", (double)v[i]);
            if (k == 0) std::fputc('\n', fp);
        };
        auto mat = [&](const float* a, int rows, int cols) {  // a is rows x cols row-major
            if (layout != GPAD_FILE_FLIPPED) {  // row-major and flat files: as stored
                for (int i = 0; i < rows; ++i) vec(a + (size_t)i * cols, cols);
            } else {
                std::vector<float> t((size_t)rows * cols);
                transpose(a, t.data(), cols, rows);  // t is cols x rows
                for (int j = 0; j < cols; ++j) vec(t.data() + (size_t)j * rows, rows);
            }
        };
        const int rows = layout == GPAD_FILE_FLAT ? f->N : n;  // flat: M_G N x m, G_L m x N
        mat(f->M_G, rows, m);
        vec(f->g_P, n);
        mat(f->G_L, m, rows);
        vec(f->p_D, m);
        vec(f->theta, f->num_iterations);
        vec(f->beta, f->num_iterations);
        const bool bad = std::ferror(fp) != 0;
        if (std::fclose(fp) != 0 || bad) return io_fail("gpad_datafile_write: write error");
        return GPAD_OK;
    });
}

}  // extern "C"
