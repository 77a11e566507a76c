// zt_zarr.cpp — Zarr V3 filesystem arrays: metadata, chunk keys, fill values, codecs.
// See zt_zarr.hpp for what this restates from zarrs and the Zarr V3 specification.
#include "zt_zarr.hpp"

#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/uio.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <mutex>

#include "../../../include/zarrs_tools_amd.h"
#include "../zt_device.hpp"

namespace zt {
namespace zarr {

namespace {

const char* kNames[] = {"bool",   "int8",   "int16",   "int32",   "int64",
                        "uint8",  "uint16", "uint32",  "uint64",  "bfloat16",
                        "float16", "float32", "float64"};

[[noreturn]] void raise(int code, const std::string& m) { throw Error(code, m); }

std::string read_file(const std::string& p, bool* exists) {
    int fd = ::open(p.c_str(), O_RDONLY);
    if (fd < 0) {
        if (errno == ENOENT && exists) { *exists = false; return {}; }
        raise(ZT_ERR_IO, "open " + p + ": " + std::strerror(errno));
    }
    struct stat st;
    if (fstat(fd, &st) != 0) { ::close(fd); raise(ZT_ERR_IO, "stat " + p); }
    std::string s((size_t)st.st_size, '\0');
    size_t got = 0;
    while (got < s.size()) {
        ssize_t n = ::read(fd, &s[got], s.size() - got);
        if (n <= 0) { ::close(fd); raise(ZT_ERR_IO, "read " + p); }
        got += (size_t)n;
    }
    ::close(fd);
    if (exists) *exists = true;
    return s;
}

void mkdirs(const std::string& dir) {
    if (dir.empty()) return;
    std::string cur;
    size_t pos = 0;
    while (pos != std::string::npos) {
        pos = dir.find('/', pos + 1);
        cur = dir.substr(0, pos);
        if (cur.empty()) continue;
        if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
            raise(ZT_ERR_IO, "mkdir " + cur + ": " + std::strerror(errno));
    }
}

void write_file(const std::string& p, const void* data, size_t n) {
    size_t slash = p.rfind('/');
    if (slash != std::string::npos) mkdirs(p.substr(0, slash));
    int fd = ::open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd < 0) raise(ZT_ERR_IO, "create " + p + ": " + std::strerror(errno));
    const char* c = static_cast<const char*>(data);
    size_t put = 0;
    while (put < n) {
        ssize_t w = ::write(fd, c + put, n - put);
        if (w <= 0) { ::close(fd); raise(ZT_ERR_IO, "write " + p + ": " + std::strerror(errno)); }
        put += (size_t)w;
    }
    ::close(fd);
}

// ---- zstd through the runtime library (no development header in this image) ----------------
struct Zstd {
    size_t (*compressBound)(size_t) = nullptr;
    size_t (*decompress)(void*, size_t, const void*, size_t) = nullptr;
    unsigned long long (*getFrameContentSize)(const void*, size_t) = nullptr;
    unsigned (*isError)(size_t) = nullptr;
    void* (*createCCtx)() = nullptr;
    size_t (*freeCCtx)(void*) = nullptr;
    size_t (*setParameter)(void*, int, int) = nullptr;
    size_t (*compress2)(void*, void*, size_t, const void*, size_t) = nullptr;
    bool ok = false;
    Zstd() {
        void* h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        compressBound = (size_t(*)(size_t))dlsym(h, "ZSTD_compressBound");
        decompress = (size_t(*)(void*, size_t, const void*, size_t))dlsym(h, "ZSTD_decompress");
        getFrameContentSize =
            (unsigned long long (*)(const void*, size_t))dlsym(h, "ZSTD_getFrameContentSize");
        isError = (unsigned (*)(size_t))dlsym(h, "ZSTD_isError");
        createCCtx = (void* (*)())dlsym(h, "ZSTD_createCCtx");
        freeCCtx = (size_t(*)(void*))dlsym(h, "ZSTD_freeCCtx");
        setParameter = (size_t(*)(void*, int, int))dlsym(h, "ZSTD_CCtx_setParameter");
        compress2 = (size_t(*)(void*, void*, size_t, const void*, size_t))dlsym(h, "ZSTD_compress2");
        ok = compressBound && decompress && getFrameContentSize && isError && createCCtx &&
             freeCCtx && setParameter && compress2;
    }
};
const Zstd& zstd() {
    static Zstd z;
    return z;
}
constexpr int kZstdCLevel = 100, kZstdChecksumFlag = 201;  // ZSTD_cParameter values

// ---- crc32c (Castagnoli), slicing table ------------------------------------------------------
uint32_t g_crc_tab[8][256];
std::once_flag g_crc_once;
void crc_init() {
    for (uint32_t i = 0; i < 256; ++i) {
        uint32_t c = i;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
        g_crc_tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
        for (int t = 1; t < 8; ++t)
            g_crc_tab[t][i] = (g_crc_tab[t - 1][i] >> 8) ^ g_crc_tab[0][g_crc_tab[t - 1][i] & 0xFF];
}

int64_t prod(const std::vector<int64_t>& v) {
    int64_t p = 1;
    for (auto x : v) p *= x;
    return p;
}

void c_strides(const std::vector<int64_t>& shape, int64_t* st) {
    int64_t s = 1;
    for (int d = (int)shape.size() - 1; d >= 0; --d) { st[d] = s; s *= shape[d]; }
}

void fill_elems(uint8_t* dst, size_t n, const uint8_t* fill, size_t esz) {
    bool zero = true;
    for (size_t b = 0; b < esz; ++b) zero = zero && fill[b] == 0;
    if (zero) { std::memset(dst, 0, n * esz); return; }
    for (size_t i = 0; i < n; ++i) std::memcpy(dst + i * esz, fill, esz);
}

void byteswap(uint8_t* p, size_t n, size_t esz) {
    if (esz <= 1) return;
    for (size_t i = 0; i < n; ++i) std::reverse(p + i * esz, p + (i + 1) * esz);
}

json::Value int_array(const std::vector<int64_t>& v) {
    json::Array a;
    for (auto x : v) a.emplace_back((int64_t)x);
    return json::Value(std::move(a));
}

std::vector<int64_t> to_ints(const json::Value& v) {
    std::vector<int64_t> out;
    for (auto& e : v.arr()) out.push_back(e.as_int());
    return out;
}


// Scatter a file's byte runs into memory (or gather memory runs into a file) with preadv /
// pwritev: the uncompressed `bytes` codec needs no staging copy between the chunk file and the
// strided row buffer. Runs are (file offset, memory pointer, length); consecutive runs whose file
// ranges touch are issued as one vectored call (<= IOV_MAX iovecs).
struct Run {
    int64_t off;
    uint8_t* mem;
    size_t len;
};

void vector_io(int fd, const std::vector<Run>& runs, bool write, const std::string& what) {
    size_t i = 0;
    std::vector<struct iovec> iov;
    while (i < runs.size()) {
        iov.clear();
        const int64_t start = runs[i].off;
        int64_t end = start;
        size_t total = 0;
        while (i < runs.size() && runs[i].off == end && iov.size() < 1024) {
            iov.push_back({runs[i].mem, runs[i].len});
            end += (int64_t)runs[i].len;
            total += runs[i].len;
            ++i;
        }
        size_t done = 0;
        size_t k = 0;
        while (done < total) {
            ssize_t n = write ? ::pwritev(fd, iov.data() + k, (int)(iov.size() - k), start + (int64_t)done)
                              : ::preadv(fd, iov.data() + k, (int)(iov.size() - k), start + (int64_t)done);
            if (n <= 0) raise(ZT_ERR_IO, (write ? "write " : "read ") + what + ": " + std::strerror(errno));
            done += (size_t)n;
            // advance over the consumed iovecs
            size_t m = (size_t)n;
            while (m > 0 && k < iov.size()) {
                if (m >= iov[k].iov_len) { m -= iov[k].iov_len; ++k; }
                else {
                    iov[k].iov_base = static_cast<uint8_t*>(iov[k].iov_base) + m;
                    iov[k].iov_len -= m;
                    m = 0;
                }
            }
        }
    }
}

// The runs of an n-D box: for every index of the outer axes, the innermost contiguous run.
void box_runs(const int64_t* box, int nd, const int64_t* file_st, int64_t file_off,
              uint8_t* mem, const int64_t* mem_st, size_t esz, std::vector<Run>& out) {
    int64_t outer = 1;
    for (int d = 0; d < nd - 1; ++d) outer *= box[d];
    out.reserve((size_t)outer);
    for (int64_t o = 0; o < outer; ++o) {
        int64_t rem = o, fo = 0, mo = 0;
        for (int d = nd - 2; d >= 0; --d) {
            int64_t i = rem % box[d];
            rem /= box[d];
            fo += i * file_st[d];
            mo += i * mem_st[d];
        }
        out.push_back({(file_off + fo) * (int64_t)esz, mem + mo * (int64_t)esz, (size_t)box[nd - 1] * esz});
    }
}

}  // namespace

int dtype_from_name(const std::string& n) {
    for (int d = 0; d <= ZT_FLOAT64; ++d)
        if (n == kNames[d]) return d;
    return -1;
}
const char* dtype_name(int d) { return d >= 0 && d <= ZT_FLOAT64 ? kNames[d] : "unknown"; }
size_t dtype_size(int d) { return zt::dtype_size(d); }

uint32_t crc32c(const uint8_t* p, size_t n) {
    std::call_once(g_crc_once, crc_init);
    uint32_t c = 0xFFFFFFFFu;
    while (n >= 8) {
        uint32_t lo, hi;
        std::memcpy(&lo, p, 4);
        std::memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = g_crc_tab[7][lo & 0xFF] ^ g_crc_tab[6][(lo >> 8) & 0xFF] ^
            g_crc_tab[5][(lo >> 16) & 0xFF] ^ g_crc_tab[4][lo >> 24] ^ g_crc_tab[3][hi & 0xFF] ^
            g_crc_tab[2][(hi >> 8) & 0xFF] ^ g_crc_tab[1][(hi >> 16) & 0xFF] ^ g_crc_tab[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = (c >> 8) ^ g_crc_tab[0][(c ^ *p++) & 0xFF];
    return c ^ 0xFFFFFFFFu;
}

bool zstd_available() { return zstd().ok; }

// ---- fill values -------------------------------------------------------------------------------

json::Value fill_json_from_double(int dtype, double v) {
    if (dtype == ZT_BOOL) return json::Value(v != 0.0);
    if (dtype >= ZT_BFLOAT16) {
        if (std::isnan(v)) return json::Value("NaN");
        if (std::isinf(v)) return json::Value(v > 0 ? "Infinity" : "-Infinity");
        return json::Value(v);
    }
    return json::Value((int64_t)v);
}

std::vector<uint8_t> fill_bytes(int dtype, const json::Value& v) {
    const size_t esz = dtype_size(dtype);
    std::vector<uint8_t> out(esz, 0);
    if (v.is_str() && v.s.size() > 2 && v.s[0] == '0' && v.s[1] == 'x') {
        // raw bits, big-endian hex of the element (Zarr V3 float fill-value encoding)
        uint64_t bits = std::strtoull(v.s.c_str() + 2, nullptr, 16);
        for (size_t b = 0; b < esz; ++b) out[b] = (uint8_t)(bits >> (8 * b));
        return out;
    }
    double d = 0.0;
    bool is_int = false;
    int64_t iv = 0;
    uint64_t uv = 0;
    if (v.kind == json::Value::Bool) d = v.b ? 1.0 : 0.0;
    else if (v.kind == json::Value::Int) { is_int = true; iv = v.i; uv = (uint64_t)v.i; d = (double)v.i; }
    else if (v.kind == json::Value::Double) d = v.d;
    else if (v.is_str()) {
        if (v.s == "NaN") d = std::nan("");
        else if (v.s == "Infinity") d = INFINITY;
        else if (v.s == "-Infinity") d = -INFINITY;
        else raise(ZT_ERR_INCOMPATIBLE_FILL_VALUE, "unsupported fill_value \"" + v.s + "\"");
    } else if (v.is_null()) {
        return out;
    } else {
        raise(ZT_ERR_INCOMPATIBLE_FILL_VALUE, "unsupported fill_value");
    }
    auto put = [&](auto x) { std::memcpy(out.data(), &x, sizeof(x)); };
    switch (dtype) {
    case ZT_BOOL: put((uint8_t)(d != 0.0)); break;
    case ZT_INT8: put((int8_t)(is_int ? iv : (int64_t)d)); break;
    case ZT_INT16: put((int16_t)(is_int ? iv : (int64_t)d)); break;
    case ZT_INT32: put((int32_t)(is_int ? iv : (int64_t)d)); break;
    case ZT_INT64: put((int64_t)(is_int ? iv : (int64_t)d)); break;
    case ZT_UINT8: put((uint8_t)(is_int ? uv : (uint64_t)d)); break;
    case ZT_UINT16: put((uint16_t)(is_int ? uv : (uint64_t)d)); break;
    case ZT_UINT32: put((uint32_t)(is_int ? uv : (uint64_t)d)); break;
    case ZT_UINT64: put((uint64_t)(is_int ? uv : (uint64_t)d)); break;
    case ZT_BFLOAT16: put(zt::f64_to_bf16_bits(d)); break;
    case ZT_FLOAT16: put(zt::f64_to_f16_bits(d)); break;
    case ZT_FLOAT32: put((float)d); break;
    case ZT_FLOAT64: put(d); break;
    default: raise(ZT_ERR_UNSUPPORTED_DATA_TYPE, "fill value for an unsupported data type");
    }
    return out;
}

// ---- bytes -> bytes codecs --------------------------------------------------------------------

std::vector<uint8_t> BytesCodec::encode(const std::vector<uint8_t>& in) const {
    if (name == "gzip") {
        z_stream zs{};
        if (deflateInit2(&zs, level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
            raise(ZT_ERR_OTHER, "gzip: deflateInit2 failed");
        std::vector<uint8_t> out(deflateBound(&zs, (uLong)in.size()) + 32);
        zs.next_in = const_cast<Bytef*>(in.data());
        zs.avail_in = (uInt)in.size();
        zs.next_out = out.data();
        zs.avail_out = (uInt)out.size();
        int rc = deflate(&zs, Z_FINISH);
        size_t n = zs.total_out;
        deflateEnd(&zs);
        if (rc != Z_STREAM_END) raise(ZT_ERR_OTHER, "gzip: deflate failed");
        out.resize(n);
        return out;
    }
    if (name == "zstd") {
        const Zstd& z = zstd();
        if (!z.ok) raise(ZT_ERR_OTHER, "zstd: libzstd.so.1 not available");
        std::vector<uint8_t> out(z.compressBound(in.size()));
        void* cctx = z.createCCtx();
        z.setParameter(cctx, kZstdCLevel, level);
        z.setParameter(cctx, kZstdChecksumFlag, checksum ? 1 : 0);
        size_t n = z.compress2(cctx, out.data(), out.size(), in.data(), in.size());
        z.freeCCtx(cctx);
        if (z.isError(n)) raise(ZT_ERR_OTHER, "zstd: compression failed");
        out.resize(n);
        return out;
    }
    if (name == "crc32c") {
        std::vector<uint8_t> out(in);
        uint32_t c = crc32c(in.data(), in.size());
        for (int b = 0; b < 4; ++b) out.push_back((uint8_t)(c >> (8 * b)));
        return out;
    }
    raise(ZT_ERR_OTHER, "unsupported codec " + name);
}

std::vector<uint8_t> BytesCodec::decode(const std::vector<uint8_t>& in, size_t expect) const {
    if (name == "gzip") {
        z_stream zs{};
        if (inflateInit2(&zs, 15 + 32) != Z_OK) raise(ZT_ERR_OTHER, "gzip: inflateInit2 failed");
        std::vector<uint8_t> out(expect ? expect : in.size() * 4 + 64);
        zs.next_in = const_cast<Bytef*>(in.data());
        zs.avail_in = (uInt)in.size();
        int rc;
        for (;;) {
            zs.next_out = out.data() + zs.total_out;
            zs.avail_out = (uInt)(out.size() - zs.total_out);
            rc = inflate(&zs, Z_FINISH);
            if (rc == Z_STREAM_END) break;
            if (rc != Z_OK && rc != Z_BUF_ERROR) { inflateEnd(&zs); raise(ZT_ERR_OTHER, "gzip: corrupt data"); }
            if (zs.avail_in == 0 && rc == Z_BUF_ERROR && zs.avail_out != 0) {
                inflateEnd(&zs);
                raise(ZT_ERR_OTHER, "gzip: truncated data");
            }
            out.resize(out.size() * 2);
        }
        out.resize(zs.total_out);
        inflateEnd(&zs);
        return out;
    }
    if (name == "zstd") {
        const Zstd& z = zstd();
        if (!z.ok) raise(ZT_ERR_OTHER, "zstd: libzstd.so.1 not available");
        unsigned long long fcs = z.getFrameContentSize(in.data(), in.size());
        size_t cap = (fcs < (1ULL << 62)) ? (size_t)fcs : (expect ? expect : in.size() * 8);
        for (;;) {
            std::vector<uint8_t> out(cap);
            size_t n = z.decompress(out.data(), out.size(), in.data(), in.size());
            if (!z.isError(n)) { out.resize(n); return out; }
            if (cap > ((size_t)1 << 40)) raise(ZT_ERR_OTHER, "zstd: decompression failed");
            cap *= 2;
        }
    }
    if (name == "crc32c") {
        if (in.size() < 4) raise(ZT_ERR_OTHER, "crc32c: short chunk");
        size_t n = in.size() - 4;
        uint32_t want = 0;
        for (int b = 0; b < 4; ++b) want |= (uint32_t)in[n + b] << (8 * b);
        if (crc32c(in.data(), n) != want) raise(ZT_ERR_OTHER, "crc32c: checksum mismatch");
        return std::vector<uint8_t>(in.begin(), in.begin() + (ptrdiff_t)n);
    }
    raise(ZT_ERR_OTHER, "unsupported codec " + name);
}

json::Value BytesCodec::to_json() const {
    json::Value cfg = json::Value(json::Object{});
    if (name == "gzip") cfg.set("level", (int64_t)level);
    if (name == "zstd") { cfg.set("level", (int64_t)level); cfg.set("checksum", checksum); }
    json::Value v = json::Value(json::Object{});
    v.set("name", name);
    if (name != "crc32c") v.set("configuration", cfg);
    return v;
}

// ---- codec chains -----------------------------------------------------------------------------

CodecChain CodecChain::from_json(const json::Value& codecs, int ndim) {
    CodecChain c;
    bool have_a2b = false;
    for (auto& cv : codecs.arr()) {
        const std::string name = cv.is_str() ? cv.s : cv.at("name").str();
        const json::Value* cfg = cv.is_obj() ? cv.find("configuration") : nullptr;
        if (name == "bytes") {
            if (have_a2b) raise(ZT_ERR_ARRAY, "two array->bytes codecs");
            have_a2b = true;
            const json::Value* e = cfg ? cfg->find("endian") : nullptr;
            c.big_endian = e && e->is_str() && e->s == "big";
        } else if (name == "sharding_indexed") {
            if (have_a2b) raise(ZT_ERR_ARRAY, "two array->bytes codecs");
            if (!cfg) raise(ZT_ERR_ARRAY, "sharding_indexed without configuration");
            have_a2b = true;
            c.sharded = true;
            c.inner_shape = to_ints(cfg->at("chunk_shape"));
            if ((int)c.inner_shape.size() != ndim)
                raise(ZT_ERR_ARRAY, "sharding chunk_shape rank mismatch");
            c.inner = std::make_shared<CodecChain>(from_json(cfg->at("codecs"), ndim));
            const json::Value* ic = cfg->find("index_codecs");
            json::Value def = json::parse(
                "[{\"name\":\"bytes\",\"configuration\":{\"endian\":\"little\"}},{\"name\":\"crc32c\"}]");
            c.index = std::make_shared<CodecChain>(from_json(ic ? *ic : def, 1));
            const json::Value* loc = cfg->find("index_location");
            c.index_at_end = !(loc && loc->is_str() && loc->s == "start");
        } else if (name == "gzip" || name == "zstd" || name == "crc32c") {
            if (!have_a2b) raise(ZT_ERR_ARRAY, "bytes->bytes codec before the array->bytes codec");
            BytesCodec b;
            b.name = name;
            if (cfg) {
                if (auto* l = cfg->find("level")) b.level = (int)l->as_int();
                if (auto* k = cfg->find("checksum")) b.checksum = k->kind == json::Value::Bool && k->b;
            }
            if (name == "zstd" && !zstd().ok)
                raise(ZT_ERR_ARRAY, "zstd codec: libzstd.so.1 not loadable");
            c.b2b.push_back(b);
        } else {
            raise(ZT_ERR_ARRAY, "unsupported codec \"" + name + "\" (supported: bytes, "
                                "sharding_indexed, gzip, zstd, crc32c)");
        }
    }
    if (!have_a2b) raise(ZT_ERR_ARRAY, "codec chain without an array->bytes codec");
    return c;
}

json::Value CodecChain::to_json() const {
    json::Array a;
    if (sharded) {
        json::Value cfg = json::Value(json::Object{});
        cfg.set("chunk_shape", int_array(inner_shape));
        cfg.set("codecs", inner->to_json());
        cfg.set("index_codecs", index->to_json());
        cfg.set("index_location", index_at_end ? "end" : "start");
        json::Value v = json::Value(json::Object{});
        v.set("name", "sharding_indexed");
        v.set("configuration", cfg);
        a.push_back(v);
    } else {
        json::Value cfg = json::Value(json::Object{});
        cfg.set("endian", big_endian ? "big" : "little");
        json::Value v = json::Value(json::Object{});
        v.set("name", "bytes");
        v.set("configuration", cfg);
        a.push_back(v);
    }
    for (auto& b : b2b) a.push_back(b.to_json());
    return json::Value(std::move(a));
}

std::vector<uint8_t> CodecChain::encode_bytes(std::vector<uint8_t> raw, size_t esz) const {
    if (big_endian) byteswap(raw.data(), raw.size() / esz, esz);
    for (auto& b : b2b) raw = b.encode(raw);
    return raw;
}

std::vector<uint8_t> CodecChain::decode_bytes(const std::vector<uint8_t>& bytes, size_t raw_bytes,
                                              size_t esz) const {
    std::vector<uint8_t> cur = bytes;
    for (int k = (int)b2b.size() - 1; k >= 0; --k) cur = b2b[k].decode(cur, k == 0 ? raw_bytes : 0);
    if (cur.size() != raw_bytes) raise(ZT_ERR_ARRAY, "decoded chunk has the wrong size");
    if (big_endian) byteswap(cur.data(), cur.size() / esz, esz);
    return cur;
}

std::vector<uint8_t> CodecChain::encode(const uint8_t* raw, const std::vector<int64_t>& shape,
                                        size_t esz, const uint8_t* fill) const {
    const int nd = (int)shape.size();
    if (!sharded) return encode_bytes(std::vector<uint8_t>(raw, raw + prod(shape) * esz), esz);
    // Shard: inner chunks in C order of the inner grid, then the (offset, nbytes) index.
    std::vector<int64_t> ig(nd), sst(nd), ist(nd);
    for (int d = 0; d < nd; ++d) ig[d] = (shape[d] + inner_shape[d] - 1) / inner_shape[d];
    c_strides(shape, sst.data());
    c_strides(inner_shape, ist.data());
    const int64_t n_inner = prod(ig), ie = prod(inner_shape);
    std::vector<uint64_t> idx((size_t)n_inner * 2);
    std::vector<uint8_t> body, tmp((size_t)ie * esz);
    std::vector<int64_t> box(nd);
    for (int64_t c = 0; c < n_inner; ++c) {
        int64_t rem = c, off = 0;
        for (int d = nd - 1; d >= 0; --d) {
            int64_t ci = rem % ig[d];
            rem /= ig[d];
            off += ci * inner_shape[d] * sst[d];
            box[d] = std::min(inner_shape[d], shape[d] - ci * inner_shape[d]);
        }
        fill_elems(tmp.data(), (size_t)ie, fill, esz);
        copy_box(raw + off * esz, sst.data(), tmp.data(), ist.data(), box.data(), nd, esz);
        std::vector<uint8_t> enc = inner->encode(tmp.data(), inner_shape, esz, fill);
        idx[2 * c] = body.size();
        idx[2 * c + 1] = enc.size();
        body.insert(body.end(), enc.begin(), enc.end());
    }
    std::vector<uint8_t> ib((size_t)n_inner * 16);
    std::memcpy(ib.data(), idx.data(), ib.size());  // little-endian host
    if (!index_at_end) {
        // offsets are relative to the shard start: shift by the encoded index size
        std::vector<uint8_t> probe = index->encode_bytes(ib, 8);
        for (int64_t c = 0; c < n_inner; ++c) idx[2 * c] += probe.size();
        std::memcpy(ib.data(), idx.data(), ib.size());
    }
    std::vector<uint8_t> ienc = index->encode_bytes(ib, 8);
    if (index_at_end) {
        body.insert(body.end(), ienc.begin(), ienc.end());
        return body;
    }
    ienc.insert(ienc.end(), body.begin(), body.end());
    return ienc;
}

void CodecChain::decode(const std::vector<uint8_t>& bytes, uint8_t* raw,
                        const std::vector<int64_t>& shape, size_t esz, const uint8_t* fill) const {
    const int nd = (int)shape.size();
    const size_t raw_bytes = (size_t)prod(shape) * esz;
    if (!sharded) {
        std::vector<uint8_t> r = decode_bytes(bytes, raw_bytes, esz);
        std::memcpy(raw, r.data(), raw_bytes);
        return;
    }
    std::vector<int64_t> ig(nd), sst(nd), ist(nd);
    for (int d = 0; d < nd; ++d) ig[d] = (shape[d] + inner_shape[d] - 1) / inner_shape[d];
    c_strides(shape, sst.data());
    c_strides(inner_shape, ist.data());
    const int64_t n_inner = prod(ig), ie = prod(inner_shape);
    // index size: 16 B per inner chunk plus what the index codecs add (crc32c: 4 B)
    size_t isz = (size_t)n_inner * 16;
    for (auto& b : index->b2b) {
        if (b.name == "crc32c") isz += 4;
        else raise(ZT_ERR_ARRAY, "sharding index codec " + b.name + " not supported");
    }
    if (bytes.size() < isz) raise(ZT_ERR_ARRAY, "shard shorter than its index");
    std::vector<uint8_t> ienc(index_at_end ? bytes.end() - (ptrdiff_t)isz : bytes.begin(),
                              index_at_end ? bytes.end() : bytes.begin() + (ptrdiff_t)isz);
    std::vector<uint8_t> ib = index->decode_bytes(ienc, (size_t)n_inner * 16, 8);
    std::vector<uint64_t> idx((size_t)n_inner * 2);
    std::memcpy(idx.data(), ib.data(), ib.size());
    std::vector<uint8_t> tmp((size_t)ie * esz);
    std::vector<int64_t> box(nd);
    for (int64_t c = 0; c < n_inner; ++c) {
        int64_t rem = c, off = 0;
        for (int d = nd - 1; d >= 0; --d) {
            int64_t ci = rem % ig[d];
            rem /= ig[d];
            off += ci * inner_shape[d] * sst[d];
            box[d] = std::min(inner_shape[d], shape[d] - ci * inner_shape[d]);
        }
        const uint64_t o = idx[2 * c], n = idx[2 * c + 1];
        if (o == ~0ULL && n == ~0ULL) {
            fill_elems(tmp.data(), (size_t)ie, fill, esz);
        } else {
            if (o + n > bytes.size()) raise(ZT_ERR_ARRAY, "shard index points past the shard");
            std::vector<uint8_t> sub(bytes.begin() + (ptrdiff_t)o, bytes.begin() + (ptrdiff_t)(o + n));
            inner->decode(sub, tmp.data(), inner_shape, esz, fill);
        }
        copy_box(tmp.data(), ist.data(), raw + off * esz, sst.data(), box.data(), nd, esz);
    }
}

// ---- strided box copy --------------------------------------------------------------------------

void copy_box(const uint8_t* src, const int64_t* ss, uint8_t* dst, const int64_t* ds,
              const int64_t* box, int nd, size_t esz) {
    for (int d = 0; d < nd; ++d)
        if (box[d] <= 0) return;
    if (nd == 0) { std::memcpy(dst, src, esz); return; }
    // innermost run (contiguous in both when the last strides are 1)
    const int64_t run = box[nd - 1];
    const bool contig = ss[nd - 1] == 1 && ds[nd - 1] == 1;
    int64_t outer = 1;
    for (int d = 0; d < nd - 1; ++d) outer *= box[d];
    for (int64_t o = 0; o < outer; ++o) {
        int64_t rem = o, so = 0, dof = 0;
        for (int d = nd - 2; d >= 0; --d) {
            int64_t i = rem % box[d];
            rem /= box[d];
            so += i * ss[d];
            dof += i * ds[d];
        }
        if (contig) {
            std::memcpy(dst + dof * esz, src + so * esz, (size_t)run * esz);
        } else {
            for (int64_t i = 0; i < run; ++i)
                std::memcpy(dst + (dof + i * ds[nd - 1]) * esz, src + (so + i * ss[nd - 1]) * esz,
                            esz);
        }
    }
}

// ---- arrays ------------------------------------------------------------------------------------

Array Array::open(const std::string& path) {
    bool exists = false;
    std::string text = read_file(path + "/zarr.json", &exists);
    // An array being written by several processes keeps its metadata under a name Zarr readers
    // do not see until the writer publishes it (renames it to zarr.json) once every chunk is in:
    // the reference's store_metadata-after-the-chunks order (zarrs_ome.rs:729), across processes.
    if (!exists) text = read_file(path + "/" + kPendingMetadata, &exists);
    if (!exists) raise(ZT_ERR_STORAGE, "no Zarr V3 array at " + path + " (zarr.json missing)");
    json::Value m;
    try {
        m = json::parse(text);
    } catch (const std::exception& e) {
        raise(ZT_ERR_JSON, path + "/zarr.json: " + e.what());
    }
    Array a;
    a.path = path;
    try {
        if (m.at("zarr_format").as_int() != 3) raise(ZT_ERR_ARRAY, "not a Zarr V3 array");
        if (m.at("node_type").str() != "array") raise(ZT_ERR_ARRAY, path + " is not an array");
        a.shape = to_ints(m.at("shape"));
        const std::string dt = m.at("data_type").is_str() ? m.at("data_type").str() : "";
        a.dtype = dtype_from_name(dt);
        if (a.dtype < 0) raise(ZT_ERR_UNSUPPORTED_DATA_TYPE, "unsupported data type " + dt);
        a.esz = dtype_size(a.dtype);
        const json::Value& grid = m.at("chunk_grid");
        if (grid.at("name").str() != "regular") raise(ZT_ERR_ARRAY, "only regular chunk grids");
        a.chunk_shape = to_ints(grid.at("configuration").at("chunk_shape"));
        if (a.chunk_shape.size() != a.shape.size()) raise(ZT_ERR_ARRAY, "chunk_shape rank mismatch");
        for (auto c : a.chunk_shape)
            if (c <= 0) raise(ZT_ERR_ARRAY, "chunk extents must be positive");
        const json::Value& ke = m.at("chunk_key_encoding");
        a.key_encoding = ke.at("name").str();
        a.separator = a.key_encoding == "v2" ? '.' : '/';
        if (const json::Value* cfg = ke.find("configuration"))
            if (const json::Value* s = cfg->find("separator")) a.separator = s->str()[0];
        if (a.key_encoding != "default" && a.key_encoding != "v2")
            raise(ZT_ERR_ARRAY, "unsupported chunk key encoding " + a.key_encoding);
        a.fill_json = m.at("fill_value");
        a.fill = fill_bytes(a.dtype, a.fill_json);
        a.codecs = CodecChain::from_json(m.at("codecs"), a.ndim());
        if (a.codecs.sharded)
            for (int d = 0; d < a.ndim(); ++d)
                if (a.chunk_shape[d] % a.codecs.inner_shape[d] != 0)
                    raise(ZT_ERR_ARRAY, "shard shape must be a multiple of the inner chunk shape");
        if (const json::Value* at = m.find("attributes")) a.attributes = *at;
        if (const json::Value* dn = m.find("dimension_names")) a.dimension_names = *dn;
    } catch (const Error&) {
        throw;
    } catch (const std::exception& e) {
        raise(ZT_ERR_ARRAY, path + "/zarr.json: " + e.what());
    }
    return a;
}

Array Array::create(const std::string& path, int dtype, const std::vector<int64_t>& shape,
                    const std::vector<int64_t>& chunk_shape, const json::Value& codecs,
                    const json::Value& fill_value) {
    if (dtype < 0 || dtype > ZT_FLOAT64) raise(ZT_ERR_UNSUPPORTED_DATA_TYPE, "bad data type");
    if (shape.size() != chunk_shape.size() || shape.empty())
        raise(ZT_ERR_INVALID_PARAMETERS, "shape / chunk_shape rank mismatch");
    for (auto c : chunk_shape)
        if (c <= 0) raise(ZT_ERR_INVALID_PARAMETERS, "chunk extents must be positive");
    Array a;
    a.path = path;
    a.shape = shape;
    a.chunk_shape = chunk_shape;
    a.dtype = dtype;
    a.esz = dtype_size(dtype);
    a.fill_json = fill_value;
    a.fill = fill_bytes(dtype, fill_value);
    a.codecs = CodecChain::from_json(
        codecs.is_null()
            ? json::parse("[{\"name\":\"bytes\",\"configuration\":{\"endian\":\"little\"}}]")
            : codecs,
        (int)shape.size());
    a.attributes = json::Value(json::Object{});
    mkdirs(path);
    return a;
}

json::Value Array::metadata() const {
    json::Value m = json::Value(json::Object{});
    m.set("zarr_format", (int64_t)3);
    m.set("node_type", "array");
    m.set("shape", int_array(shape));
    m.set("data_type", dtype_name(dtype));
    json::Value gc = json::Value(json::Object{});
    gc.set("chunk_shape", int_array(chunk_shape));
    json::Value grid = json::Value(json::Object{});
    grid.set("name", "regular");
    grid.set("configuration", gc);
    m.set("chunk_grid", grid);
    json::Value kc = json::Value(json::Object{});
    kc.set("separator", std::string(1, separator));
    json::Value ke = json::Value(json::Object{});
    ke.set("name", key_encoding);
    ke.set("configuration", kc);
    m.set("chunk_key_encoding", ke);
    m.set("fill_value", fill_json);
    m.set("codecs", codecs.to_json());
    m.set("attributes", attributes.is_null() ? json::Value(json::Object{}) : attributes);
    if (!dimension_names.is_null()) m.set("dimension_names", dimension_names);
    return m;
}

void Array::store_metadata() const {
    std::string s = json::dump(metadata(), 2) + "\n";
    write_file(path + "/zarr.json", s.data(), s.size());
}

void Array::erase_metadata() const { ::unlink((path + "/zarr.json").c_str()); }

std::vector<int64_t> Array::grid_shape() const {
    std::vector<int64_t> g(shape.size());
    for (size_t d = 0; d < shape.size(); ++d)
        g[d] = (shape[d] + chunk_shape[d] - 1) / chunk_shape[d];
    return g;
}

std::string Array::chunk_key(const int64_t* idx) const {
    std::string k;
    if (key_encoding == "default") {
        k = "c";
        for (int d = 0; d < ndim(); ++d) { k += separator; k += std::to_string(idx[d]); }
    } else {
        for (int d = 0; d < ndim(); ++d) {
            if (d) k += separator;
            k += std::to_string(idx[d]);
        }
        if (ndim() == 0) k = "0";
    }
    return k;
}

int64_t Array::chunk_elems() const { return prod(chunk_shape); }

size_t Array::read_chunk(const int64_t* idx, uint8_t* dst, const int64_t* dst_origin,
                         const int64_t* dst_shape, const int64_t* dst_strides) const {
    const int nd = ndim();
    // the part of the chunk inside the array and the destination region
    std::vector<int64_t> lo(nd), box(nd), cst(nd);
    for (int d = 0; d < nd; ++d) {
        const int64_t c0 = idx[d] * chunk_shape[d];
        const int64_t a = std::max(c0, dst_origin[d]);
        const int64_t b = std::min({c0 + chunk_shape[d], shape[d], dst_origin[d] + dst_shape[d]});
        lo[d] = a;
        box[d] = b - a;
        if (box[d] <= 0) return 0;
    }
    c_strides(chunk_shape, cst.data());
    int64_t doff = 0, soff = 0;
    for (int d = 0; d < nd; ++d) {
        doff += (lo[d] - dst_origin[d]) * dst_strides[d];
        soff += (lo[d] - idx[d] * chunk_shape[d]) * cst[d];
    }
    const bool raw_codec = !codecs.sharded && codecs.b2b.empty() && !codecs.big_endian;
    if (raw_codec && dst_strides[nd - 1] == 1) {
        // uncompressed: scatter the needed runs of the file straight into the destination
        const std::string p = chunk_path(idx);
        int fd = ::open(p.c_str(), O_RDONLY);
        if (fd >= 0) {
            struct stat stt;
            if (fstat(fd, &stt) != 0 || (size_t)stt.st_size != (size_t)chunk_elems() * esz) {
                ::close(fd);
                raise(ZT_ERR_ARRAY, p + ": chunk has the wrong size");
            }
            std::vector<Run> runs;
            box_runs(box.data(), nd, cst.data(), soff, dst + doff * esz, dst_strides, esz, runs);
            try {
                vector_io(fd, runs, false, p);
            } catch (...) {
                ::close(fd);
                throw;
            }
            ::close(fd);
            int64_t n = 1;
            for (int d = 0; d < nd; ++d) n *= box[d];
            return (size_t)n * esz;
        }
        if (errno != ENOENT) raise(ZT_ERR_IO, "open " + p + ": " + std::strerror(errno));
    }
    bool exists = false;
    std::string enc = raw_codec && dst_strides[nd - 1] == 1 ? std::string() : read_file(chunk_path(idx), &exists);
    if (!exists) {
        // missing chunk: the fill value over the region
        std::vector<int64_t> zero(nd, 0);
        std::vector<uint8_t> f(esz);
        std::memcpy(f.data(), fill.data(), esz);
        int64_t outer = 1;
        for (int d = 0; d < nd; ++d) outer *= box[d];
        std::vector<uint8_t> tmp((size_t)outer * esz);
        fill_elems(tmp.data(), (size_t)outer, fill.data(), esz);
        std::vector<int64_t> tst(nd);
        c_strides(box, tst.data());
        copy_box(tmp.data(), tst.data(), dst + doff * esz, dst_strides, box.data(), nd, esz);
        return 0;
    }
    std::vector<uint8_t> bytes(enc.begin(), enc.end());
    std::string().swap(enc);
    if (!codecs.sharded && codecs.b2b.empty() && !codecs.big_endian) {
        // bytes codec only: the file is the chunk
        if (bytes.size() != (size_t)chunk_elems() * esz)
            raise(ZT_ERR_ARRAY, chunk_path(idx) + ": chunk has the wrong size");
        copy_box(bytes.data() + soff * esz, cst.data(), dst + doff * esz, dst_strides, box.data(),
                 nd, esz);
        return bytes.size();
    }
    std::vector<uint8_t> raw((size_t)chunk_elems() * esz);
    codecs.decode(bytes, raw.data(), chunk_shape, esz, fill.data());
    copy_box(raw.data() + soff * esz, cst.data(), dst + doff * esz, dst_strides, box.data(), nd,
             esz);
    return bytes.size();
}

size_t Array::write_chunk(const int64_t* idx, const uint8_t* src, const int64_t* src_origin,
                          const int64_t* src_shape, const int64_t* src_strides) const {
    const int nd = ndim();
    std::vector<int64_t> lo(nd), box(nd), cst(nd);
    bool full = true;
    for (int d = 0; d < nd; ++d) {
        const int64_t c0 = idx[d] * chunk_shape[d];
        const int64_t b = std::min(c0 + chunk_shape[d], shape[d]);
        if (c0 < src_origin[d] || b > src_origin[d] + src_shape[d])
            raise(ZT_ERR_INVALID_PARAMETERS, "write_chunk: region does not cover the chunk");
        lo[d] = c0;
        box[d] = b - c0;
        full = full && box[d] == chunk_shape[d];
    }
    c_strides(chunk_shape, cst.data());
    int64_t soff = 0;
    for (int d = 0; d < nd; ++d) soff += (lo[d] - src_origin[d]) * src_strides[d];
    const bool raw_codec = !codecs.sharded && codecs.b2b.empty() && !codecs.big_endian;
    if (raw_codec && full && src_strides[nd - 1] == 1) {
        // uncompressed full chunk: gather the runs of the source straight into the file
        const std::string p = chunk_path(idx);
        size_t slash = p.rfind('/');
        if (slash != std::string::npos) mkdirs(p.substr(0, slash));
        int fd = ::open(p.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) raise(ZT_ERR_IO, "create " + p + ": " + std::strerror(errno));
        std::vector<Run> runs;
        box_runs(box.data(), nd, cst.data(), 0, const_cast<uint8_t*>(src) + soff * esz, src_strides,
                 esz, runs);
        try {
            vector_io(fd, runs, true, p);
        } catch (...) {
            ::close(fd);
            throw;
        }
        ::close(fd);
        return (size_t)chunk_elems() * esz;
    }
    std::vector<uint8_t> raw((size_t)chunk_elems() * esz);
    if (!full) fill_elems(raw.data(), (size_t)chunk_elems(), fill.data(), esz);
    copy_box(src + soff * esz, src_strides, raw.data(), cst.data(), box.data(), nd, esz);
    std::vector<uint8_t> enc =
        (!codecs.sharded && codecs.b2b.empty() && !codecs.big_endian)
            ? std::move(raw)
            : codecs.encode(raw.data(), chunk_shape, esz, fill.data());
    write_file(chunk_path(idx), enc.data(), enc.size());
    return enc.size();
}

}  // namespace zarr
}  // namespace zt
