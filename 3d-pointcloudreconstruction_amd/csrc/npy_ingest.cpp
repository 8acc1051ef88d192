// npy_ingest.cpp -- batched ground-truth cloud ingestion.
//
// Reference: every training/eval sample loads its ground truth with
// np.load(data_dir_pcl + model + '/pointcloud_' + str(numpoints) + '.npy')
// (utils/datasets_old.py:37-38), one file per __getitem__, collated by the
// DataLoader and copied to the GPU with .cuda() (train.py:152-156).
//
// Here one call reads a whole batch of .npy clouds straight into the caller's
// (pinned) [count, npoints, 3] float32 buffer with a pool of threads; the host
// side then issues ONE asynchronous copy to HBM (utils/gt_ingest.py).  Host
// code only: no device work, no allocation beyond per-thread read buffers.
//
// Accepted files: NPY format 1.0 / 2.0 / 3.0, descr '<f4' '>f4' '<f8' '>f8'
// (also '=' / '|' byte order marks), C or Fortran order, shape (npoints, 3).
// Values are converted to float32 exactly as numpy's astype(np.float32)
// (round to nearest even).
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

#include "pcm.h"

namespace {

struct NpyHeader {
    int elem = 0;          // 4 or 8
    bool big = false;      // big-endian payload
    bool fortran = false;  // column-major
    long rows = -1, cols = -1;
    long data_offset = 0;
};

// Parse "{'descr': '<f4', 'fortran_order': False, 'shape': (1024, 3), }".
bool parse_dict(const std::string &h, NpyHeader &out) {
    auto value_after = [&](const char *key) -> size_t {
        const size_t k = h.find(key);
        if (k == std::string::npos) return std::string::npos;
        const size_t c = h.find(':', k + strlen(key));
        if (c == std::string::npos) return std::string::npos;
        size_t v = c + 1;
        while (v < h.size() && h[v] == ' ') ++v;
        return v;
    };
    size_t v = value_after("'descr'");
    if (v == std::string::npos || v + 4 > h.size() || (h[v] != '\'' && h[v] != '"')) return false;
    const char q = h[v];
    const size_t e = h.find(q, v + 1);
    if (e == std::string::npos) return false;
    const std::string d = h.substr(v + 1, e - v - 1);
    if (d.size() != 3 || d[1] != 'f') return false;
    if (d[0] == '<' || d[0] == '=' || d[0] == '|') out.big = false;
    else if (d[0] == '>') out.big = true;
    else return false;
    if (d[2] == '4') out.elem = 4;
    else if (d[2] == '8') out.elem = 8;
    else return false;
    v = value_after("'fortran_order'");
    if (v == std::string::npos) return false;
    if (h.compare(v, 4, "True") == 0) out.fortran = true;
    else if (h.compare(v, 5, "False") == 0) out.fortran = false;
    else return false;
    v = value_after("'shape'");
    if (v == std::string::npos || h[v] != '(') return false;
    long dims[2] = {-1, -1};
    int nd = 0;
    size_t p = v + 1;
    while (p < h.size() && h[p] != ')') {
        while (p < h.size() && (h[p] == ' ' || h[p] == ',')) ++p;
        if (p < h.size() && h[p] >= '0' && h[p] <= '9') {
            long x = 0;
            while (p < h.size() && h[p] >= '0' && h[p] <= '9') x = x * 10 + (h[p++] - '0');
            if (nd >= 2) return false;  // not a 2-D array
            dims[nd++] = x;
        } else if (p < h.size() && h[p] != ')') {
            return false;
        }
    }
    if (nd != 2) return false;
    out.rows = dims[0];
    out.cols = dims[1];
    return true;
}

// Parse the NPY preamble + header dict at the start of `p` (n bytes).
int parse_header(const unsigned char *p, size_t n, NpyHeader &hd) {
    if (n < 10) return PCM_ERR_IO;
    if (memcmp(p, "\x93NUMPY", 6) != 0) return PCM_ERR_FORMAT;
    const int major = p[6];
    uint32_t hlen;
    size_t off;
    if (major == 1) {
        hlen = (uint32_t)p[8] | ((uint32_t)p[9] << 8);
        off = 10;
    } else if (major == 2 || major == 3) {
        if (n < 12) return PCM_ERR_IO;
        hlen = (uint32_t)p[8] | ((uint32_t)p[9] << 8) | ((uint32_t)p[10] << 16) | ((uint32_t)p[11] << 24);
        off = 12;
    } else {
        return PCM_ERR_FORMAT;
    }
    if (hlen > (1u << 20)) return PCM_ERR_FORMAT;
    if (off + hlen > n) return PCM_ERR_IO;
    if (!parse_dict(std::string((const char *)p + off, hlen), hd)) return PCM_ERR_FORMAT;
    hd.data_offset = (long)(off + hlen);
    return PCM_OK;
}

// Whole file into buf (one read for the usual ~12 KB cloud).
int slurp(const char *path, std::vector<unsigned char> &buf, size_t &n) {
    const int fd = open(path, O_RDONLY | O_CLOEXEC);
    if (fd < 0) return PCM_ERR_IO;
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size < 0) { close(fd); return PCM_ERR_IO; }
    n = (size_t)st.st_size;
    if (buf.size() < n) buf.resize(n);
    size_t got = 0;
    while (got < n) {
        const ssize_t r = read(fd, buf.data() + got, n - got);
        if (r <= 0) break;
        got += (size_t)r;
    }
    close(fd);
    return got == n ? PCM_OK : PCM_ERR_IO;
}

inline uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
inline uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// One file -> out[npoints * 3] (row-major float32).  buf: per-thread scratch.
int load_one(const char *path, int npoints, float *out, std::vector<unsigned char> &buf) {
    size_t n = 0;
    int rc = slurp(path, buf, n);
    if (rc != PCM_OK) return rc;
    NpyHeader hd;
    rc = parse_header(buf.data(), n, hd);
    if (rc != PCM_OK) return rc;
    if (hd.rows != npoints || hd.cols != 3) return PCM_ERR_FORMAT;
    const size_t count = (size_t)npoints * 3;
    if ((size_t)hd.data_offset + count * hd.elem > n) return PCM_ERR_IO;  // truncated
    const unsigned char *data = buf.data() + hd.data_offset;
    if (hd.elem == 4 && !hd.big && !hd.fortran) {  // the common case: little-endian float32, C order
        memcpy(out, data, count * 4);
        return PCM_OK;
    }
    for (size_t i = 0; i < count; ++i) {
        // element i of the file's memory order -> (row, col)
        size_t r, c;
        if (hd.fortran) { c = i / (size_t)npoints; r = i % (size_t)npoints; }
        else { r = i / 3; c = i % 3; }
        float v;
        if (hd.elem == 4) {
            uint32_t b;
            memcpy(&b, data + 4 * i, 4);
            if (hd.big) b = bswap32(b);
            memcpy(&v, &b, 4);
        } else {
            uint64_t b;
            memcpy(&b, data + 8 * i, 8);
            if (hd.big) b = bswap64(b);
            double dv;
            memcpy(&dv, &b, 8);
            v = (float)dv;  // IEEE round to nearest even, as numpy's astype
        }
        out[r * 3 + c] = v;
    }
    return PCM_OK;
}

}  // namespace

extern "C" int pcm_npy_cloud_points(const char *path, int *npoints) {
    if (!path || !npoints) return PCM_ERR_INVALID_ARG;
    std::vector<unsigned char> buf;
    size_t n = 0;
    int rc = slurp(path, buf, n);
    if (rc != PCM_OK) return rc;
    NpyHeader hd;
    rc = parse_header(buf.data(), n, hd);
    if (rc != PCM_OK) return rc;
    if (hd.cols != 3 || hd.rows < 0 || hd.rows > 0x7fffffff) return PCM_ERR_FORMAT;
    *npoints = (int)hd.rows;
    return PCM_OK;
}

extern "C" int pcm_npy_load_clouds(const char *const *paths, int count, int npoints, float *out, int nthreads,
                                   int *failed_index) {
    if (failed_index) *failed_index = -1;
    if (count < 0 || npoints < 0 || (count > 0 && (!paths || !out))) return PCM_ERR_INVALID_ARG;
    if (count == 0) return PCM_OK;
    // a thread costs ~20 us to start, a warm-cache file ~5 us to read: give
    // each thread at least 8 files
    if (nthreads > (count + 7) / 8) nthreads = (count + 7) / 8;
    if (nthreads < 1) nthreads = 1;
    std::atomic<int> next{0};
    std::atomic<int> first_bad{count};
    std::atomic<int> bad_rc{PCM_OK};
    auto worker = [&]() {
        std::vector<unsigned char> buf;
        for (;;) {
            const int i = next.fetch_add(1);
            if (i >= count) break;
            const int rc = paths[i] ? load_one(paths[i], npoints, out + (size_t)i * npoints * 3, buf)
                                    : PCM_ERR_INVALID_ARG;
            if (rc != PCM_OK) {
                // keep the lowest failing index (deterministic report)
                int cur = first_bad.load();
                while (i < cur && !first_bad.compare_exchange_weak(cur, i)) {
                }
                if (first_bad.load() == i) bad_rc.store(rc);
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(worker);
    worker();
    for (auto &th : pool) th.join();
    if (first_bad.load() < count) {
        if (failed_index) *failed_index = first_bad.load();
        // re-derive the code of the lowest failing file (bad_rc may belong to a later one)
        std::vector<unsigned char> buf;
        std::vector<float> tmp((size_t)npoints * 3);
        const int i = first_bad.load();
        const int rc = paths[i] ? load_one(paths[i], npoints, tmp.data(), buf) : PCM_ERR_INVALID_ARG;
        return rc != PCM_OK ? rc : bad_rc.load();
    }
    return PCM_OK;
}
