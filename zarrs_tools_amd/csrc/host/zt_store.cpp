// zt_store.cpp — the store -> store path: Zarr V3 arrays on host storage in, Zarr V3 arrays out,
// the per-chunk transform on the GPU in between (C ABI: include/zarrs_tools_amd.h, "store").
//
// Reference: GuidedFilter::apply / apply_chunk (guided_filter.rs:75-114, 240-319) read every
// output chunk's 2r-halo subset from the input store (decoding up to 3^d input chunks per output
// chunk), filter it on a rayon worker, and store the output chunk; zarrs_ome's level loop
// (zarrs_ome.rs:515-738) does the same with Downsample. Here the chunk grid is walked in chunk
// rows along axis 0, and the work is pipelined over host threads and three HIP streams:
//
//   decode row j+1.. (host pool)  |  H2D slab k -> kernel k -> D2H row k (GPU)  |  encode row k-1
//
// Each input chunk is decoded exactly once into a pinned host row buffer (a ring of rows); the
// slab for output row k = the planes [z0 - 2r, z1 + 2r) is assembled on the device from the rows
// that hold them, so the halo is shared instead of re-decoded. Output rows come back into a
// double-buffered pinned host buffer and are encoded chunk by chunk on the pool.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <exception>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/zarrs_tools_amd.h"
#include "../zt_device.hpp"
#include "zt_zarr.hpp"

namespace zt {
int set_last_error(int code, const char* msg);
}

namespace {

using zt::zarr::Array;
using Clock = std::chrono::steady_clock;

double secs_since(Clock::time_point t0) {
    return std::chrono::duration<double>(Clock::now() - t0).count();
}

// ---- a small fixed thread pool with task groups ------------------------------------------------
class Group {
  public:
    void add() {
        std::lock_guard<std::mutex> l(m_);
        ++pending_;
    }
    void done(std::exception_ptr e) {
        std::lock_guard<std::mutex> l(m_);
        if (e && !err_) err_ = e;
        if (--pending_ == 0) cv_.notify_all();
    }
    void wait() {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return pending_ == 0; });
        if (err_) {
            std::exception_ptr e = err_;
            err_ = nullptr;
            std::rethrow_exception(e);
        }
    }
    void wait_nothrow() {
        std::unique_lock<std::mutex> l(m_);
        cv_.wait(l, [&] { return pending_ == 0; });
    }

  private:
    std::mutex m_;
    std::condition_variable cv_;
    int pending_ = 0;
    std::exception_ptr err_;
};

class Pool {
  public:
    explicit Pool(int n) {
        for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void submit(Group& g, std::function<void()> f) {
        g.add();
        {
            std::lock_guard<std::mutex> l(m_);
            q_.emplace_back([&g, f = std::move(f)] {
                std::exception_ptr e;
                try {
                    f();
                } catch (...) {
                    e = std::current_exception();
                }
                g.done(e);
            });
        }
        cv_.notify_one();
    }
    int size() const { return (int)th_.size(); }

  private:
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> l(m_);
                cv_.wait(l, [&] { return stop_ || !q_.empty(); });
                if (stop_ && q_.empty()) return;
                f = std::move(q_.front());
                q_.pop_front();
            }
            f();
        }
    }
    std::vector<std::thread> th_;
    std::deque<std::function<void()>> q_;
    std::mutex m_;
    std::condition_variable cv_;
    bool stop_ = false;
};

int resolve_threads(int n) {
    if (n > 0) return n;
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc ? hc : 8u, 16u));
}

std::vector<int64_t> c_strides(const std::vector<int64_t>& shape) {
    std::vector<int64_t> st(shape.size());
    int64_t s = 1;
    for (int d = (int)shape.size() - 1; d >= 0; --d) { st[d] = s; s *= shape[d]; }
    return st;
}

// every chunk index of the chunk rows [r0, r1) along axis 0
// Chunks of rows [r0, r1) along axis 0 whose axis-1 index lies in [c0, c1) (c1 < 0: all).
std::vector<std::vector<int64_t>> chunks_in_rows(const Array& a, int64_t r0, int64_t r1,
                                                 int64_t c0 = 0, int64_t c1 = -1) {
    const auto g = a.grid_shape();
    const int nd = a.ndim();
    int64_t per = 1;
    for (int d = 1; d < nd; ++d) per *= g[d];
    std::vector<std::vector<int64_t>> out;
    for (int64_t r = r0; r < r1; ++r)
        for (int64_t c = 0; c < per; ++c) {
            std::vector<int64_t> idx(nd);
            idx[0] = r;
            int64_t rem = c;
            for (int d = nd - 1; d >= 1; --d) { idx[d] = rem % g[d]; rem /= g[d]; }
            if (nd > 1 && c1 >= 0 && (idx[1] < c0 || idx[1] >= c1)) continue;
            out.push_back(idx);
        }
    return out;
}

// An output window along axis 1 (config T's (t, z) block split): output elements [o0, o1) and
// the input elements [i0, i1) they read (the halo, clamped). Absent: the whole axis.
struct ColWin {
    int64_t o0, o1, i0, i1;
};

struct Pinned {
    void* p = nullptr;
    size_t n = 0;
    void alloc(size_t bytes) {
        n = bytes;
        if (bytes && hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            throw zt::zarr::Error(ZT_ERR_OUT_OF_MEMORY, "pinned host allocation failed");
        }
    }
    ~Pinned() {
        if (p) (void)hipHostFree(p);
    }
    uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

struct DevBuf {
    void* p = nullptr;
    void alloc(size_t bytes) {
        if (bytes && hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            p = nullptr;
            throw zt::zarr::Error(ZT_ERR_OUT_OF_MEMORY, "device allocation failed");
        }
    }
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
    uint8_t* u8() const { return static_cast<uint8_t*>(p); }
};

#define HIPCHK(x)                                                                                \
    do {                                                                                         \
        hipError_t _e = (x);                                                                     \
        if (_e != hipSuccess)                                                                    \
            throw zt::zarr::Error(ZT_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct Events {
    std::vector<hipEvent_t> ev;
    hipEvent_t make() {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        ev.push_back(e);
        return e;
    }
    ~Events() {
        for (auto e : ev) (void)hipEventDestroy(e);
    }
};

struct Streams {
    std::vector<hipStream_t> s;
    hipStream_t make() {
        hipStream_t x;
        HIPCHK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
        s.push_back(x);
        return x;
    }
    ~Streams() {
        for (auto x : s) {
            (void)hipStreamSynchronize(x);
            (void)hipStreamDestroy(x);
        }
    }
};

struct Ctx {
    zt_ctx* c = nullptr;
    ~Ctx() {
        if (c) zt_ctx_destroy(c);
    }
};

float ev_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
        (void)hipGetLastError();
        return 0.f;
    }
    return ms;
}

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ULL;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
    return x ^ (x >> 31);
}

// Convert a fill value to another data type with Rust `as` semantics (convert_fill_value,
// lib.rs:836-899, num_traits::AsPrimitive): float -> int saturates (NaN -> 0) and truncates
// toward zero, int -> int wraps, anything -> float rounds to nearest.
zt::json::Value convert_fill(const Array& a, int dtype_out) {
    const uint8_t* f = a.fill.data();
    bool is_float = false, is_signed = false;
    double v = 0.0;
    int64_t iv = 0;
    uint64_t uv = 0;
    switch (a.dtype) {
    case ZT_BOOL: case ZT_UINT8: uv = f[0]; break;
    case ZT_INT8: iv = (int8_t)f[0]; is_signed = true; break;
    case ZT_INT16: { int16_t x; std::memcpy(&x, f, 2); iv = x; is_signed = true; break; }
    case ZT_INT32: { int32_t x; std::memcpy(&x, f, 4); iv = x; is_signed = true; break; }
    case ZT_INT64: { int64_t x; std::memcpy(&x, f, 8); iv = x; is_signed = true; break; }
    case ZT_UINT16: { uint16_t x; std::memcpy(&x, f, 2); uv = x; break; }
    case ZT_UINT32: { uint32_t x; std::memcpy(&x, f, 4); uv = x; break; }
    case ZT_UINT64: { std::memcpy(&uv, f, 8); break; }
    case ZT_BFLOAT16: { uint16_t x; std::memcpy(&x, f, 2); v = zt::bf16_bits_to_f32(x); is_float = true; break; }
    case ZT_FLOAT16: { uint16_t x; std::memcpy(&x, f, 2); v = zt::f16_bits_to_f32(x); is_float = true; break; }
    case ZT_FLOAT32: { float x; std::memcpy(&x, f, 4); v = x; is_float = true; break; }
    case ZT_FLOAT64: std::memcpy(&v, f, 8); is_float = true; break;
    }
    if (!is_float) {
        if (is_signed) uv = (uint64_t)iv;
        v = is_signed ? (double)iv : (double)uv;
    }
    if (dtype_out >= ZT_BFLOAT16) return zt::zarr::fill_json_from_double(dtype_out, v);
    // integer (and bool, as u8) targets
    int bits = 8;
    bool sgn = false;
    switch (dtype_out) {
    case ZT_INT8: sgn = true; bits = 8; break;
    case ZT_INT16: sgn = true; bits = 16; break;
    case ZT_INT32: sgn = true; bits = 32; break;
    case ZT_INT64: sgn = true; bits = 64; break;
    case ZT_UINT16: bits = 16; break;
    case ZT_UINT32: bits = 32; break;
    case ZT_UINT64: bits = 64; break;
    default: bits = 8; break;  // bool, uint8
    }
    uint64_t out;
    if (is_float) {  // saturating
        if (std::isnan(v)) out = 0;
        else if (sgn) {
            const double lo = -std::ldexp(1.0, bits - 1), hi = std::ldexp(1.0, bits - 1);
            const double t = std::trunc(v);
            out = t <= lo ? (uint64_t)(int64_t)lo : t >= hi ? (uint64_t)((int64_t)(hi - 1 >= 9.2e18 ? INT64_MAX : (int64_t)hi - 1))
                                                         : (uint64_t)(int64_t)t;
        } else {
            const double hi = std::ldexp(1.0, bits);
            const double t = std::trunc(v);
            out = t <= 0 ? 0 : t >= hi ? (bits == 64 ? UINT64_MAX : (uint64_t)hi - 1) : (uint64_t)t;
        }
    } else {
        out = uv;  // wrapping
    }
    if (bits < 64) out &= ((uint64_t)1 << bits) - 1;
    if (dtype_out == ZT_BOOL) return zt::json::Value(out != 0);
    if (sgn) {
        int64_t sv = (int64_t)(out << (64 - bits)) >> (64 - bits);  // sign-extend
        return zt::json::Value(sv);
    }
    return zt::json::Value((uint64_t)out);
}

// ---- the output array of a filter: FilterTraits::output_array_builder (filter_traits.rs:47-82)
//      + get_array_builder_reencode (lib.rs:408-650) ---------------------------------------------
//
// `enc` is a JSON object with ZarrReencodingArgs' keys (lib.rs:274-377): data_type, fill_value,
// separator, chunk_shape, shard_shape, array_to_array_codecs, array_to_bytes_codec,
// bytes_to_bytes_codecs, dimension_names, attributes, attributes_append; absent keys keep the
// input's. Restated as the reference computes it, quirks included:
//  * the base is the input array (shape, chunk grid, key encoding, attributes, dimension names);
//  * an unsharded input's base "chunk shape" is its chunk GRID shape (lib.rs:447), and a chunk
//    shape (override or base) only takes effect when the output is sharded: without a shard
//    shape the output keeps the input's chunk grid (lib.rs:623-646);
//  * shard = min(shard, input extent) (0 = the input extent), rounded up to a multiple of the
//    chunk shape; chunk 0 = the input extent (lib.rs:462-494);
//  * a new data type without a fill value converts the input fill value (`as` semantics).
// Codecs supported here: bytes, gzip, zstd, crc32c, sharding_indexed (no array -> array codecs).
Array build_output(const Array& in, const std::string& out_path, int dtype_filter,
                   const std::vector<int64_t>& out_shape, const char* enc_json) {
    using zt::json::Value;
    Value enc = (enc_json && *enc_json) ? zt::json::parse(enc_json) : Value(zt::json::Object{});
    if (!enc.is_obj())
        throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS, "encoding: a JSON object expected");
    static const char* known[] = {"data_type", "fill_value", "separator", "chunk_shape",
                                  "shard_shape", "array_to_array_codecs", "array_to_bytes_codec",
                                  "bytes_to_bytes_codecs", "dimension_names", "attributes",
                                  "attributes_append"};
    for (const auto& kv : *enc.o) {
        bool ok = false;
        for (const char* k : known) ok = ok || kv.first == k;
        if (!ok) throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS, "encoding: unknown key " + kv.first);
    }
    const int nd = in.ndim();
    auto ints = [&](const Value& v, const char* what) {
        std::vector<int64_t> r;
        if (!v.is_arr() || (int)v.arr().size() != nd)
            throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS,
                                  std::string("encoding: ") + what + " needs one entry per axis");
        for (const auto& x : v.arr()) r.push_back(x.as_int());
        return r;
    };
    // base: the input's chunk / shard shapes and codec chain (lib.rs:414-458)
    std::vector<int64_t> chunk, shard;
    bool sharded = false;
    zt::zarr::CodecChain chain;  // the (inner) chain: bytes + b2b
    if (in.codecs.sharded) {
        chunk = in.codecs.inner_shape;
        shard = in.chunk_shape;
        sharded = true;
        chain = *in.codecs.inner;
    } else {
        chunk = in.grid_shape();
        chain = in.codecs;
    }
    if (const Value* c = enc.find("chunk_shape")) {
        chunk = ints(*c, "chunk_shape");
        for (int d = 0; d < nd; ++d) if (chunk[d] == 0) chunk[d] = in.shape[d];
    }
    if (const Value* sv = enc.find("shard_shape")) {
        shard = ints(*sv, "shard_shape");
        for (int d = 0; d < nd; ++d) shard[d] = shard[d] == 0 ? in.shape[d] : std::min(shard[d], in.shape[d]);
        sharded = true;
    }
    if (sharded)
        for (int d = 0; d < nd; ++d) {
            if (chunk[d] <= 0) throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS, "encoding: chunk extents must be positive");
            shard[d] = (shard[d] + chunk[d] - 1) / chunk[d] * chunk[d];  // next_multiple_of
        }
    if (const Value* a2a = enc.find("array_to_array_codecs")) {
        const Value v = a2a->is_str() ? zt::json::parse(a2a->str()) : *a2a;
        if (!v.is_arr() || !v.arr().empty())
            throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS,
                                  "encoding: array to array codecs are not supported on this path");
    }
    // the chain JSON [array_to_bytes, bytes_to_bytes...], overrides applied
    Value inner_js = chain.to_json();
    Value a2b = inner_js.arr().at(0);
    std::vector<Value> b2b(inner_js.arr().begin() + 1, inner_js.arr().end());
    if (const Value* v = enc.find("array_to_bytes_codec")) a2b = v->is_str() ? zt::json::parse(v->str()) : *v;
    if (const Value* v = enc.find("bytes_to_bytes_codecs")) {
        const Value l = v->is_str() ? zt::json::parse(v->str()) : *v;
        if (!l.is_arr()) throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS, "encoding: bytes_to_bytes_codecs must be a list");
        b2b = l.arr();
    }
    zt::json::Array inner_list{a2b};
    for (auto& c : b2b) inner_list.push_back(c);
    Value codecs;
    std::vector<int64_t> grid_chunk;
    if (sharded) {
        Value cfg = Value(zt::json::Object{});
        cfg.set("chunk_shape", Value([&] { zt::json::Array a; for (auto c : chunk) a.push_back(Value(c)); return a; }()));
        cfg.set("codecs", Value(inner_list));
        cfg.set("index_codecs", zt::json::parse(
            "[{\"name\":\"bytes\",\"configuration\":{\"endian\":\"little\"}},{\"name\":\"crc32c\"}]"));
        cfg.set("index_location", "end");
        Value sh = Value(zt::json::Object{});
        sh.set("name", "sharding_indexed");
        sh.set("configuration", cfg);
        codecs = Value(zt::json::Array{sh});
        grid_chunk = shard;
    } else {
        codecs = Value(inner_list);
        grid_chunk = in.chunk_shape;  // the builder keeps the input's chunk grid
    }
    // data type and fill value (filter_traits.rs:53-74, lib.rs:585-611)
    int dt = in.dtype;
    bool dt_changed = false;
    if (const Value* v = enc.find("data_type")) {
        dt = zt::zarr::dtype_from_name(v->str());
        if (dt < 0) throw zt::zarr::Error(ZT_ERR_UNSUPPORTED_DATA_TYPE, "unsupported data type " + v->str());
        dt_changed = true;
    } else if (dtype_filter >= 0 && dtype_filter != in.dtype) {
        dt = dtype_filter;
        dt_changed = true;
    }
    Value fill = in.fill_json;
    if (const Value* v = enc.find("fill_value")) fill = *v;
    else if (dt_changed) fill = convert_fill(in, dt);
    Array out = Array::create(out_path, dt, out_shape, grid_chunk, codecs, fill);
    out.key_encoding = in.key_encoding;
    out.separator = in.separator;
    if (const Value* v = enc.find("separator")) {
        const std::string sep = v->str();
        if (sep != "/" && sep != ".")
            throw zt::zarr::Error(ZT_ERR_INVALID_PARAMETERS, "encoding: separator must be / or .");
        out.key_encoding = "default";  // chunk_key_encoding_default_separator (lib.rs:585-587)
        out.separator = sep[0];
    }
    out.attributes = in.attributes.is_null() ? Value(zt::json::Object{}) : in.attributes;
    if (const Value* v = enc.find("attributes")) out.attributes = v->is_str() ? zt::json::parse(v->str()) : *v;
    if (const Value* v = enc.find("attributes_append")) {
        const Value add = v->is_str() ? zt::json::parse(v->str()) : *v;
        if (add.is_obj()) for (const auto& kv : *add.o) out.attributes.set(kv.first, kv.second);
    }
    out.dimension_names = in.dimension_names;
    if (const Value* v = enc.find("dimension_names")) out.dimension_names = *v;
    return out;
}

int report(const std::exception& e) {
    if (auto* z = dynamic_cast<const zt::zarr::Error*>(&e)) return zt::set_last_error(z->code, z->what());
    return zt::set_last_error(ZT_ERR_OTHER, e.what());
}

// ---- the chunk-row pipeline --------------------------------------------------------------------

// What one output chunk row needs from the input and how it is computed on the device.
// ---- calculate_chunk_limit (filter.rs:52-66) for the row pipeline ------------------------------
// The reference bounds the chunks in flight by 80 % of the available RAM / memory_per_chunk and
// fails with FilterError::Other when not even one chunk fits. Here the unit in flight is a chunk
// row (pinned host rows, device slabs): the ring depth and double buffering are chosen from 80 %
// of the available host RAM and 80 % of the free device memory, down to one row without overlap,
// and the reference's error is returned when not even that fits. ZT_STORE_HOST_MEMORY /
// ZT_STORE_DEVICE_MEMORY (bytes) override the available amounts (tests, co-tenant limits).
// One unsigned number from a cgroup file; false when absent or "max" (no limit).
bool read_cgroup_u64(const char* path, uint64_t& v) {
    FILE* f = std::fopen(path, "r");
    if (!f) return false;
    char buf[64] = {0};
    const bool got = std::fgets(buf, sizeof buf, f) != nullptr;
    std::fclose(f);
    if (!got || buf[0] < '0' || buf[0] > '9') return false;
    v = std::strtoull(buf, nullptr, 10);
    return true;
}

// "key value" from a cgroup memory.stat file.
bool read_stat_key(const std::string& path, const char* key, uint64_t& v) {
    FILE* f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    char line[256];
    bool found = false;
    const size_t kl = std::strlen(key);
    while (std::fgets(line, sizeof line, f)) {
        if (std::strncmp(line, key, kl) == 0 && line[kl] == ' ') {
            v = std::strtoull(line + kl + 1, nullptr, 10);
            found = true;
            break;
        }
    }
    std::fclose(f);
    return found;
}

uint64_t host_available_bytes() {
    if (const char* e = std::getenv("ZT_STORE_HOST_MEMORY")) return std::strtoull(e, nullptr, 10);
    // ZT_MEMINFO / ZT_CGROUP_ROOT relocate the files read below (tests)
    const char* mi = std::getenv("ZT_MEMINFO");
    FILE* f = std::fopen(mi ? mi : "/proc/meminfo", "r");
    uint64_t kb = 0;
    if (f) {
        char line[256];
        while (std::fgets(line, sizeof line, f))
            if (std::sscanf(line, "MemAvailable: %lu kB", (unsigned long*)&kb) == 1) break;
        std::fclose(f);
    }
    uint64_t avail = kb ? kb * 1024 : (uint64_t)16 << 30;
    // Inside a memory-limited cgroup MemAvailable describes the whole machine: cap it at the
    // cgroup's limit minus its usage (v2: memory.max / memory.current, v1: limit / usage). The
    // usage counts page cache, which the kernel reclaims on demand (a store pipeline that has just
    // read or written GBs of chunks sits near its limit on cache alone), so the inactive file
    // pages (memory.stat inactive_file / total_inactive_file) are subtracted from it, as
    // MemAvailable counts reclaimable cache as available.
    const char* cr = std::getenv("ZT_CGROUP_ROOT");
    const std::string root = cr ? cr : "/sys/fs/cgroup";
    uint64_t lim = 0, use = 0, inact = 0;
    bool got = false;
    if (read_cgroup_u64((root + "/memory.max").c_str(), lim) &&
        read_cgroup_u64((root + "/memory.current").c_str(), use)) {
        got = true;
        if (!read_stat_key(root + "/memory.stat", "inactive_file", inact)) inact = 0;
    } else if (read_cgroup_u64((root + "/memory/memory.limit_in_bytes").c_str(), lim) &&
               read_cgroup_u64((root + "/memory/memory.usage_in_bytes").c_str(), use)) {
        got = true;
        if (!read_stat_key(root + "/memory/memory.stat", "total_inactive_file", inact)) inact = 0;
    }
    if (got && lim < ((uint64_t)1 << 60)) {
        const uint64_t used = use > inact ? use - inact : 0;
        avail = std::min(avail, lim > used ? lim - used : 0);
    }
    return avail;
}

// --chunk-limit (zarrs_ome.rs:136-141, guided_filter.rs:251-258): the reference processes at
// most this many chunks concurrently. Per calling thread; 0 = bounded by memory only.
thread_local int64_t g_chunk_limit = 0;

uint64_t device_available_bytes() {
    if (const char* e = std::getenv("ZT_STORE_DEVICE_MEMORY")) return std::strtoull(e, nullptr, 10);
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return fr;
}

const char* kNotEnoughMemory =
    "There is not enough available memory to process a single output chunk. Consider reducing "
    "the chunk shape (or shard shape if sharding)";

// ---- progress (Progress / ProgressCallback, progress.rs:15-119) ---------------------------------
std::mutex g_progress_mu;
zt_progress_fn g_progress_fn = nullptr;
void* g_progress_user = nullptr;

struct RowOp {
    // device scratch the transform allocates for a slab of `planes` input planes (estimate)
    std::function<uint64_t(int64_t planes)> scratch_bytes;
    // input planes along axis 0 for output planes [z0, z1)
    std::function<void(int64_t z0, int64_t z1, int64_t& in0, int64_t& in1)> input_planes;
    // run the transform: slab (input planes [in0, in1)) -> out (output planes [z0, z1))
    std::function<int(zt_ctx*, const void* slab, int64_t in0, int64_t in1, void* out, int64_t z0,
                      int64_t z1)>
        apply;
};

void run_pipeline(const Array& in, const Array& out, int device, int64_t row_begin,
                  int64_t row_end, int nthreads, const RowOp& op, zt_store_stats* st,
                  const ColWin* cw = nullptr) {
    const auto t_start = Clock::now();
    const int nd = in.ndim();
    const int64_t in_cz = in.chunk_shape[0], out_cz = out.chunk_shape[0];
    const int64_t nz_in = in.shape[0], nz_out = out.shape[0];
    const int64_t out_rows = (nz_out + out_cz - 1) / out_cz;
    row_begin = std::max<int64_t>(0, row_begin);
    row_end = row_end < 0 ? out_rows : std::min(row_end, out_rows);
    if (row_begin >= row_end) return;
    int64_t in_plane = 1, out_plane = 1;
    for (int d = 1; d < nd; ++d) in_plane *= (cw && d == 1) ? cw->i1 - cw->i0 : in.shape[d];
    for (int d = 1; d < out.ndim(); ++d) out_plane *= (cw && d == 1) ? cw->o1 - cw->o0 : out.shape[d];
    // chunk index ranges of the window along axis 1
    const int64_t ic0 = cw ? cw->i0 / in.chunk_shape[1] : 0;
    const int64_t ic1 = cw ? (cw->i1 + in.chunk_shape[1] - 1) / in.chunk_shape[1] : -1;
    const int64_t oc0 = cw ? cw->o0 / out.chunk_shape[1] : 0;
    const int64_t oc1 = cw ? (cw->o1 + out.chunk_shape[1] - 1) / out.chunk_shape[1] : -1;
    const size_t in_pb = (size_t)in_plane * in.esz, out_pb = (size_t)out_plane * out.esz;

    // input row span of each output row, and the largest slab
    auto span = [&](int64_t k, int64_t& in0, int64_t& in1, int64_t& j0, int64_t& j1) {
        const int64_t z0 = k * out_cz, z1 = std::min(z0 + out_cz, nz_out);
        op.input_planes(z0, z1, in0, in1);
        j0 = in0 / in_cz;
        j1 = (in1 - 1) / in_cz;
    };
    int64_t max_slab = 0, max_rows_per = 1;
    for (int64_t k = row_begin; k < row_end; ++k) {
        int64_t a, b, j0, j1;
        span(k, a, b, j0, j1);
        max_slab = std::max(max_slab, b - a);
        max_rows_per = std::max(max_rows_per, j1 - j0 + 1);
    }
    // memory budget: ring depth NR (rows decoded ahead) and NB (double-buffered slabs / outputs)
    const uint64_t in_row_b = (uint64_t)in_cz * in_pb, out_row_b = (uint64_t)out_cz * out_pb;
    const uint64_t host_budget = host_available_bytes() / 10 * 8;
    int64_t NR = max_rows_per + 2;  // ring of decoded input rows (+1 decoding ahead, +1 slack)
    int NB = 2;
    while (NR * in_row_b + (uint64_t)NB * out_row_b > host_budget) {
        if (NR > max_rows_per) --NR;
        else if (NB > 1) NB = 1;
        else throw zt::zarr::Error(ZT_ERR_OUT_OF_MEMORY, kNotEnoughMemory);
    }
    // --chunk-limit: the chunks held in flight (decoded input rows + output rows being computed
    // or encoded) stay within the limit, down to the pipeline's unit of one slab and one output
    // row without overlap (a chunk row is the device's unit of work)
    const int64_t in_row_chunks = (int64_t)chunks_in_rows(in, 0, 1, ic0, ic1).size();
    const int64_t out_row_chunks = (int64_t)chunks_in_rows(out, 0, 1, oc0, oc1).size();
    int threads = resolve_threads(nthreads);
    if (g_chunk_limit > 0) {
        while (NR * in_row_chunks + NB * out_row_chunks > g_chunk_limit) {
            if (NR > max_rows_per) --NR;
            else if (NB > 1) NB = 1;
            else break;
        }
        threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, g_chunk_limit));
    }

    if (hipSetDevice(device) != hipSuccess)
        throw zt::zarr::Error(ZT_ERR_DEVICE, "hipSetDevice failed");
    {
        const uint64_t scratch = op.scratch_bytes ? op.scratch_bytes(max_slab) : 0;
        const uint64_t dev_budget = device_available_bytes() / 10 * 8;
        auto dev_need = [&](int nb) {
            return (uint64_t)nb * ((uint64_t)max_slab * in_pb + out_row_b) + scratch;
        };
        if (dev_need(NB) > dev_budget) NB = 1;
        if (dev_need(NB) > dev_budget) throw zt::zarr::Error(ZT_ERR_OUT_OF_MEMORY, kNotEnoughMemory);
    }
    Ctx ctx;
    if (int rc = zt_ctx_create(device, &ctx.c)) throw zt::zarr::Error(rc, zt_last_error());
    Streams streams;
    hipStream_t s_h2d = streams.make(), s_comp = streams.make(), s_d2h = streams.make();
    if (int rc = zt_ctx_set_stream(ctx.c, s_comp)) throw zt::zarr::Error(rc, zt_last_error());
    Events E;
    hipEvent_t ev_h2d0[2], ev_h2d[2], ev_k0[2], ev_k[2], ev_d2h0[2], ev_d2h[2];
    for (int s = 0; s < 2; ++s) {
        ev_h2d0[s] = E.make(); ev_h2d[s] = E.make(); ev_k0[s] = E.make(); ev_k[s] = E.make();
        ev_d2h0[s] = E.make(); ev_d2h[s] = E.make();
    }
    std::vector<hipEvent_t> ring_ev(NR);
    std::vector<bool> ring_ev_set(NR, false);
    for (auto& e : ring_ev) e = E.make();

    std::vector<Pinned> hin(NR);
    for (auto& h : hin) h.alloc((size_t)in_cz * in_pb);
    Pinned hout[2];
    for (int s = 0; s < NB; ++s) hout[s].alloc((size_t)out_cz * out_pb);
    DevBuf dslab[2], dout[2];
    for (int s = 0; s < NB; ++s) {
        dslab[s].alloc((size_t)max_slab * in_pb);
        dout[s].alloc((size_t)out_cz * out_pb);
    }

    Pool pool(threads);
    std::vector<Group> dec_group(NR);
    Group enc_group[2];
    std::vector<int64_t> ring_row(NR, -1);
    std::atomic<uint64_t> bytes_read{0}, bytes_written{0};
    std::atomic<int64_t> dec_ns{0}, enc_ns{0}, k_us{0}, chunks_done{0};
    double h2d_ms = 0, k_ms = 0, d2h_ms = 0;
    int64_t chunks_total = 0;
    for (int64_t k = row_begin; k < row_end; ++k)
        chunks_total += (int64_t)chunks_in_rows(out, k, k + 1, oc0, oc1).size();

    // region descriptors of a host row buffer (C order, in_cz planes; the axis-1 window)
    std::vector<int64_t> in_row_shape(in.shape);
    in_row_shape[0] = in_cz;
    if (cw) in_row_shape[1] = cw->i1 - cw->i0;
    const std::vector<int64_t> in_row_st = c_strides(in_row_shape);
    std::vector<int64_t> out_row_shape(out.shape);
    out_row_shape[0] = out_cz;
    if (cw) out_row_shape[1] = cw->o1 - cw->o0;
    const std::vector<int64_t> out_row_st = c_strides(out_row_shape);

    auto submit_decode = [&](int64_t j) {
        const int64_t s = j % NR;
        if (ring_row[s] >= 0) {
            dec_group[s].wait();
            if (ring_ev_set[s]) HIPCHK(hipEventSynchronize(ring_ev[s]));  // H2D done reading it
        }
        ring_row[s] = j;
        uint8_t* buf = hin[s].u8();
        for (auto& idx : chunks_in_rows(in, j, j + 1, ic0, ic1)) {
            pool.submit(dec_group[s], [&, idx, buf, j] {
                const auto t0 = Clock::now();
                std::vector<int64_t> origin(nd, 0);
                origin[0] = j * in_cz;
                if (cw) origin[1] = cw->i0;
                size_t n = in.read_chunk(idx.data(), buf, origin.data(), in_row_shape.data(),
                                         in_row_st.data());
                bytes_read += n;
                dec_ns += (int64_t)(secs_since(t0) * 1e9);
            });
        }
    };
    auto submit_encode = [&](int64_t k) {
        const int s = (int)(k % NB);
        uint8_t* buf = hout[s].u8();
        for (auto& idx : chunks_in_rows(out, k, k + 1, oc0, oc1)) {
            pool.submit(enc_group[s], [&, idx, buf, k] {
                const auto t0 = Clock::now();
                std::vector<int64_t> origin(out.ndim(), 0);
                origin[0] = k * out_cz;
                if (cw) origin[1] = cw->o0;
                size_t n = out.write_chunk(idx.data(), buf, origin.data(), out_row_shape.data(),
                                           out_row_st.data());
                bytes_written += n;
                enc_ns += (int64_t)(secs_since(t0) * 1e9);
                std::lock_guard<std::mutex> lk(g_progress_mu);
                const int64_t step = ++chunks_done;  // Progress::next (progress.rs:101-104)
                if (g_progress_fn) {
                    zt_progress pr{};
                    pr.step = step;
                    pr.num_steps = chunks_total;
                    pr.read_s = dec_ns.load() * 1e-9;
                    pr.process_s = k_us.load() * 1e-6;
                    pr.write_s = enc_ns.load() * 1e-9;
                    g_progress_fn(&pr, g_progress_user);
                }
            });
        }
    };

    int64_t next_dec;
    {
        int64_t a, b, j0, j1;
        span(row_begin, a, b, j0, j1);
        next_dec = j0;
    }
    const int64_t in_rows_total = (nz_in + in_cz - 1) / in_cz;
    int64_t pending_enc = -1;  // output row whose D2H is queued but not yet handed to the encoders
    auto finish_row = [&](int64_t k) {
        const int s = (int)(k % NB);
        HIPCHK(hipEventSynchronize(ev_d2h[s]));
        h2d_ms += ev_ms(ev_h2d0[s], ev_h2d[s]);
        const float km = ev_ms(ev_k0[s], ev_k[s]);
        k_ms += km;
        k_us += (int64_t)(km * 1e3f);
        d2h_ms += ev_ms(ev_d2h0[s], ev_d2h[s]);
        submit_encode(k);
    };
    try {
        for (int64_t k = row_begin; k < row_end; ++k) {
            int64_t in0, in1, j0, j1;
            span(k, in0, in1, j0, j1);
            int64_t nj0 = j1 + 1, nj1 = j1 + 1;  // rows of the next output row (lookahead)
            if (k + 1 < row_end) {
                int64_t a, b;
                span(k + 1, a, b, nj0, nj1);
            }
            const int64_t want = std::min(std::max(j1, nj1), in_rows_total - 1);
            while (next_dec <= want && next_dec - NR < j0) submit_decode(next_dec++);
            for (int64_t j = j0; j <= j1; ++j) dec_group[j % NR].wait();
            const int s = (int)(k % NB);
            if (NB == 1 && pending_enc >= 0) {  // single buffer: row k-1 is encoded first
                finish_row(pending_enc);
                pending_enc = -1;
            }
            enc_group[s].wait();  // host output buffer s is free again (row k-NB encoded)
            // H2D: the slab's planes from the ring rows that hold them
            HIPCHK(hipStreamWaitEvent(s_h2d, ev_k[s], 0));  // kernel k-NB no longer reads slab s
            HIPCHK(hipEventRecord(ev_h2d0[s], s_h2d));
            for (int64_t j = j0; j <= j1; ++j) {
                const int64_t p0 = std::max(in0, j * in_cz), p1 = std::min(in1, (j + 1) * in_cz);
                HIPCHK(hipMemcpyAsync(dslab[s].u8() + (size_t)(p0 - in0) * in_pb,
                                      hin[j % NR].u8() + (size_t)(p0 - j * in_cz) * in_pb,
                                      (size_t)(p1 - p0) * in_pb, hipMemcpyHostToDevice, s_h2d));
            }
            HIPCHK(hipEventRecord(ev_h2d[s], s_h2d));
            for (int64_t j = j0; j <= j1; ++j) {
                HIPCHK(hipEventRecord(ring_ev[j % NR], s_h2d));
                ring_ev_set[j % NR] = true;
            }
            // kernel
            HIPCHK(hipStreamWaitEvent(s_comp, ev_h2d[s], 0));
            HIPCHK(hipStreamWaitEvent(s_comp, ev_d2h[s], 0));  // D2H k-NB done with dout[s]
            HIPCHK(hipEventRecord(ev_k0[s], s_comp));
            const int64_t z0 = k * out_cz, z1 = std::min(z0 + out_cz, nz_out);
            if (int rc = op.apply(ctx.c, dslab[s].p, in0, in1, dout[s].p, z0, z1))
                throw zt::zarr::Error(rc, zt_last_error());
            HIPCHK(hipEventRecord(ev_k[s], s_comp));
            // D2H
            HIPCHK(hipStreamWaitEvent(s_d2h, ev_k[s], 0));
            HIPCHK(hipEventRecord(ev_d2h0[s], s_d2h));
            HIPCHK(hipMemcpyAsync(hout[s].u8(), dout[s].p, (size_t)(z1 - z0) * out_pb,
                                  hipMemcpyDeviceToHost, s_d2h));
            HIPCHK(hipEventRecord(ev_d2h[s], s_d2h));
            if (pending_enc >= 0) finish_row(pending_enc);
            pending_enc = k;
        }
        if (pending_enc >= 0) finish_row(pending_enc);
        enc_group[0].wait();
        enc_group[1].wait();
        for (auto& g : dec_group) g.wait();
    } catch (...) {
        for (auto& g : dec_group) g.wait_nothrow();
        enc_group[0].wait_nothrow();
        enc_group[1].wait_nothrow();
        (void)hipDeviceSynchronize();
        throw;
    }
    if (st) {
        st->wall_s = secs_since(t_start);
        st->decode_s = dec_ns.load() * 1e-9;
        st->encode_s = enc_ns.load() * 1e-9;
        st->h2d_s = h2d_ms * 1e-3;
        st->kernel_s = k_ms * 1e-3;
        st->d2h_s = d2h_ms * 1e-3;
        st->bytes_read = bytes_read.load();
        st->bytes_written = bytes_written.load();
        int64_t vox = 0;
        for (int64_t k = row_begin; k < row_end; ++k)
            vox += (std::min((k + 1) * out_cz, nz_out) - k * out_cz) * out_plane;
        st->voxels = (uint64_t)vox;
        st->rows = row_end - row_begin;
        st->threads = pool.size();
        st->rows_in_flight = (int)NR;
        st->double_buffered = NB == 2;
    }
}

}  // namespace

extern "C" {

int zt_store_array_info(const char* path, int* dtype, int* ndim, int64_t* shape,
                        int64_t* chunk_shape, int64_t* inner_chunk_shape) {
    try {
        if (!path) return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null path");
        Array a = Array::open(path);
        if (dtype) *dtype = a.dtype;
        if (ndim) *ndim = a.ndim();
        for (int d = 0; d < a.ndim() && d < ZT_MAX_DIMS; ++d) {
            if (shape) shape[d] = a.shape[d];
            if (chunk_shape) chunk_shape[d] = a.chunk_shape[d];
            if (inner_chunk_shape)
                inner_chunk_shape[d] = a.codecs.sharded ? a.codecs.inner_shape[d] : a.chunk_shape[d];
        }
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_create_array(const char* path, int dtype, int ndim, const int64_t* shape,
                          const int64_t* chunk_shape, const char* codecs_json,
                          const char* fill_value_json) {
    try {
        if (!path || !shape || !chunk_shape || ndim < 1 || ndim > ZT_MAX_DIMS)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "bad array description");
        zt::json::Value codecs = codecs_json ? zt::json::parse(codecs_json) : zt::json::Value();
        zt::json::Value fill =
            fill_value_json ? zt::json::parse(fill_value_json) : zt::json::Value((int64_t)0);
        if (!fill_value_json && dtype == ZT_BOOL) fill = zt::json::Value(false);
        if (!fill_value_json && dtype >= ZT_BFLOAT16) fill = zt::json::Value(0.0);
        Array a = Array::create(path, dtype, std::vector<int64_t>(shape, shape + ndim),
                                std::vector<int64_t>(chunk_shape, chunk_shape + ndim), codecs,
                                fill);
        a.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_read_subset(const char* path, const int64_t* start, const int64_t* shape,
                         void* host_out, int nthreads) {
    try {
        if (!path || !start || !shape || !host_out)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null argument");
        Array a = Array::open(path);
        const int nd = a.ndim();
        std::vector<int64_t> st(start, start + nd), sh(shape, shape + nd);
        for (int d = 0; d < nd; ++d)
            if (st[d] < 0 || sh[d] < 0 || st[d] + sh[d] > a.shape[d])
                return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "subset outside the array");
        const auto strides = c_strides(sh);
        std::vector<int64_t> c0(nd), c1(nd);
        int64_t n = 1;
        for (int d = 0; d < nd; ++d) {
            if (sh[d] == 0) return ZT_OK;
            c0[d] = st[d] / a.chunk_shape[d];
            c1[d] = (st[d] + sh[d] - 1) / a.chunk_shape[d] + 1;
            n *= c1[d] - c0[d];
        }
        Pool pool(resolve_threads(nthreads));
        Group g;
        uint8_t* dst = static_cast<uint8_t*>(host_out);
        for (int64_t c = 0; c < n; ++c) {
            std::vector<int64_t> idx(nd);
            int64_t rem = c;
            for (int d = nd - 1; d >= 0; --d) {
                idx[d] = c0[d] + rem % (c1[d] - c0[d]);
                rem /= c1[d] - c0[d];
            }
            pool.submit(g, [&, idx] { a.read_chunk(idx.data(), dst, st.data(), sh.data(), strides.data()); });
        }
        g.wait();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_write_subset(const char* path, const int64_t* start, const int64_t* shape,
                          const void* host_in, int nthreads) {
    try {
        if (!path || !start || !shape || !host_in)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null argument");
        Array a = Array::open(path);
        const int nd = a.ndim();
        std::vector<int64_t> st(start, start + nd), sh(shape, shape + nd);
        std::vector<int64_t> c0(nd), c1(nd);
        int64_t n = 1;
        for (int d = 0; d < nd; ++d) {
            if (st[d] < 0 || sh[d] < 0 || st[d] + sh[d] > a.shape[d])
                return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "subset outside the array");
            if (st[d] % a.chunk_shape[d] != 0 ||
                ((st[d] + sh[d]) % a.chunk_shape[d] != 0 && st[d] + sh[d] != a.shape[d]))
                return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS,
                                          "write subset must be chunk aligned");
            if (sh[d] == 0) return ZT_OK;
            c0[d] = st[d] / a.chunk_shape[d];
            c1[d] = (st[d] + sh[d] - 1) / a.chunk_shape[d] + 1;
            n *= c1[d] - c0[d];
        }
        const auto strides = c_strides(sh);
        Pool pool(resolve_threads(nthreads));
        Group g;
        const uint8_t* src = static_cast<const uint8_t*>(host_in);
        for (int64_t c = 0; c < n; ++c) {
            std::vector<int64_t> idx(nd);
            int64_t rem = c;
            for (int d = nd - 1; d >= 0; --d) {
                idx[d] = c0[d] + rem % (c1[d] - c0[d]);
                rem /= c1[d] - c0[d];
            }
            pool.submit(g, [&, idx] { a.write_chunk(idx.data(), src, st.data(), sh.data(), strides.data()); });
        }
        g.wait();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_write_synth(const char* path, int kind, uint64_t seed, int nthreads) {
    try {
        if (!path) return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null path");
        Array a = Array::open(path);
        if ((kind == 0 && a.dtype != ZT_FLOAT32) || (kind == 1 && a.dtype != ZT_UINT16) ||
            kind < 0 || kind > 1)
            return zt::set_last_error(ZT_ERR_UNSUPPORTED_DATA_TYPE,
                                      "synthetic kind 0 needs float32, kind 1 uint16");
        const int nd = a.ndim();
        const auto g = a.grid_shape();
        int64_t n = 1;
        for (auto x : g) n *= x;
        const auto astr = c_strides(a.shape);
        const int64_t nx = a.shape[nd - 1];
        Pool pool(resolve_threads(nthreads));
        Group grp;
        for (int64_t c = 0; c < n; ++c) {
            pool.submit(grp, [&, c] {
                std::vector<int64_t> idx(nd), org(nd), box(nd);
                int64_t rem = c;
                for (int d = nd - 1; d >= 0; --d) { idx[d] = rem % g[d]; rem /= g[d]; }
                int64_t cnt = 1;
                for (int d = 0; d < nd; ++d) {
                    org[d] = idx[d] * a.chunk_shape[d];
                    box[d] = std::min(a.chunk_shape[d], a.shape[d] - org[d]);
                    cnt *= box[d];
                }
                std::vector<uint8_t> buf((size_t)cnt * a.esz);
                const auto bst = c_strides(box);
                for (int64_t i = 0; i < cnt; ++i) {
                    int64_t r = i, gl = 0, x = 0;
                    for (int d = nd - 1; d >= 0; --d) {
                        int64_t p = org[d] + r % box[d];
                        r /= box[d];
                        gl += p * astr[d];
                        if (d == nd - 1) x = p;
                    }
                    const uint64_t h = splitmix64(seed ^ (uint64_t)gl);
                    if (kind == 0) {
                        // same rounding as the device generator: RN(100*U) then + 500 (one RN)
                        const float U = (float)(h >> 40) * (1.0f / 16777216.0f);
                        volatile float t = 100.0f * U;
                        const float v = t + (x >= nx / 2 ? 500.0f : 0.0f);
                        std::memcpy(&buf[(size_t)i * 4], &v, 4);
                    } else {
                        const uint16_t v = (uint16_t)(((h >> 40) * 65535ull) >> 24);
                        std::memcpy(&buf[(size_t)i * 2], &v, 2);
                    }
                }
                a.write_chunk(idx.data(), buf.data(), org.data(), box.data(), bst.data());
            });
        }
        grp.wait();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_create_output_like(const char* in_path, const char* out_path, int dtype_out,
                                const char* encoding_json) {
    try {
        if (!in_path || !out_path) return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null path");
        Array in = Array::open(in_path);
        Array out = build_output(in, out_path, dtype_out, in.shape, encoding_json);
        out.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_create_output(const char* in_path, const char* out_path, int dtype_out,
                           const int64_t* out_shape, int ndim, const char* encoding_json) {
    try {
        if (!in_path || !out_path) return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null path");
        Array in = Array::open(in_path);
        std::vector<int64_t> shape = in.shape;
        if (out_shape) {
            if (ndim != in.ndim())
                return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "output rank != input rank");
            for (int d = 0; d < ndim; ++d) {
                if (out_shape[d] < 0)
                    return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "negative output extent");
                shape[d] = out_shape[d];
            }
        }
        Array out = build_output(in, out_path, dtype_out, shape, encoding_json);
        out.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_guided_filter(const char* in_path, const char* out_path, int dtype_out,
                           const char* encoding_json, float epsilon, int radius, int device,
                           int64_t row_begin, int64_t row_end, int nthreads, int flags,
                           zt_store_stats* stats) {
    return zt_store_guided_filter_box(in_path, out_path, dtype_out, encoding_json, epsilon,
                                      radius, device, row_begin, row_end, 0, -1, nthreads, flags,
                                      stats);
}

int zt_store_guided_filter_box(const char* in_path, const char* out_path, int dtype_out,
                               const char* encoding_json, float epsilon, int radius, int device,
                               int64_t row_begin, int64_t row_end, int64_t col_begin,
                               int64_t col_end, int nthreads, int flags, zt_store_stats* stats) {
    try {
        if (!in_path || !out_path) return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null path");
        if (radius < 0 || radius > 127)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "radius must be in [0, 127]");
        Array in = Array::open(in_path);
        // output_array_builder: the input's shape, with the reencoding overrides and data type
        // (filter_traits.rs:47-82, lib.rs:408-650)
        Array out = build_output(in, out_path, dtype_out, in.shape, encoding_json);
        const int dt = out.dtype;
        if (int rc = zt_guided_filter_is_compatible(in.dtype, dt)) return rc;
        if (flags & ZT_STORE_ERASE_OUTPUT_METADATA) out.erase_metadata();  // "not finished" marker
        const int nd = in.ndim();
        const int64_t halo = (int64_t)((radius * 2) & 0xFF);  // u8 arithmetic (guided_filter.rs:92)
        const int64_t nz = in.shape[0];
        RowOp op;
        op.input_planes = [&](int64_t z0, int64_t z1, int64_t& a, int64_t& b) {
            a = std::max<int64_t>(0, z0 - halo);
            b = std::min(nz, z1 + halo);
        };
        const std::vector<int64_t> shape = in.shape, chunk = in.chunk_shape;
        const int din = in.dtype;
        int64_t plane = 1;
        for (int d = 1; d < nd; ++d) plane *= shape[d];
        // an output window of chunk columns along axis 1 (config T's (t, z) blocks,
        // shard.block_assignment): its input carries the halo along axis 1 too
        ColWin win{};
        const bool windowed = nd >= 2 && col_end >= 0;
        op.scratch_bytes = [&, windowed](int64_t planes) -> uint64_t {
            // separable path (n-D, r > 8, or a column window, which apply takes through
            // apply_ndarray's separable form): 5 f32 words per slab voxel; fused path: f32
            // staging of non-direct element types
            return (uint64_t)planes * plane * ((nd == 3 && radius <= 8 && !windowed) ? 8 : 20);
        };
        if (windowed) {
            const int64_t oc = out.chunk_shape[1], n1 = in.shape[1];
            const int64_t ncol = (out.shape[1] + oc - 1) / oc;
            const int64_t c0 = std::max<int64_t>(0, col_begin), c1 = std::min(col_end, ncol);
            if (c0 >= c1) return ZT_OK;
            win.o0 = c0 * oc;
            win.o1 = std::min(c1 * oc, out.shape[1]);
            win.i0 = std::max<int64_t>(0, win.o0 - halo);
            win.i1 = std::min(n1, win.o1 + halo);
            plane = plane / n1 * (win.i1 - win.i0);
        }
        op.apply = [&](zt_ctx* c, const void* slab, int64_t in0, int64_t in1, void* o, int64_t z0,
                       int64_t z1) -> int {
            if (nd == 3 && radius <= 8 && !windowed)
                return zt_guided_filter_apply_slab(c, din, slab, dt, o, shape.data(), in0,
                                                   in1 - in0, z0, z1 - z0, chunk.data(), epsilon,
                                                   radius);
            // n-D (or a window): the slab is a block whose windows clamp exactly where the
            // array's do (it carries the halo or reaches the edge on every cut axis), so
            // apply_ndarray on it is the chunked result
            std::vector<int64_t> bshape(shape), ostart(nd, 0), oshape(shape);
            bshape[0] = in1 - in0;
            ostart[0] = z0 - in0;
            oshape[0] = z1 - z0;
            if (windowed) {
                bshape[1] = win.i1 - win.i0;
                ostart[1] = win.o0 - win.i0;
                oshape[1] = win.o1 - win.o0;
            }
            return zt_guided_filter_apply_ndarray(c, din, slab, bshape.data(), nullptr, nd,
                                                  ostart.data(), oshape.data(), dt, o, nullptr,
                                                  epsilon, radius);
        };
        run_pipeline(in, out, device, row_begin, row_end, nthreads, op, stats,
                     windowed ? &win : nullptr);
        if (flags & ZT_STORE_FINISH_OUTPUT) out.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_downsample(const char* in_path, const char* out_path, const int64_t* stride,
                        int discrete, int dtype_out, const char* encoding_json, int device,
                        int64_t row_begin, int64_t row_end, int nthreads, int flags,
                        zt_store_stats* stats) {
    try {
        if (!in_path || !out_path || !stride)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null argument");
        Array in = Array::open(in_path);
        const int nd = in.ndim();
        std::vector<int64_t> st(stride, stride + nd), oshape(nd), win(nd);
        if (int rc = zt_downsample_output_shape(in.shape.data(), nd, st.data(), oshape.data()))
            return rc;
        for (int d = 0; d < nd; ++d) win[d] = std::min(st[d], in.shape[d]);
        // Downsample::output_array_builder: the output shape with the reencoding overrides
        // (zarrs_ome passes its per-level chunk / shard shapes here, zarrs_ome.rs:528-560)
        Array out = build_output(in, out_path, dtype_out, oshape, encoding_json);
        const int dt = out.dtype;
        if (int rc = zt_downsample_is_compatible(in.dtype, dt, discrete)) return rc;
        if (flags & ZT_STORE_ERASE_OUTPUT_METADATA) out.erase_metadata();
        const int din = in.dtype;
        const int64_t w0 = win[0];
        RowOp op;
        op.input_planes = [&](int64_t z0, int64_t z1, int64_t& a, int64_t& b) {
            a = z0 * w0;
            b = std::min(z1 * w0, in.shape[0]);  // input_subset (downsample.rs:64-70)
        };
        const std::vector<int64_t> ishape = in.shape;
        op.apply = [&](zt_ctx* c, const void* slab, int64_t in0, int64_t in1, void* o, int64_t z0,
                       int64_t z1) -> int {
            std::vector<int64_t> bshape(ishape);
            bshape[0] = in1 - in0;
            return zt_downsample_apply_ndarray(c, din, slab, bshape.data(), nd, st.data(),
                                               discrete, dt, o);
        };
        run_pipeline(in, out, device, row_begin, row_end, nthreads, op, stats);
        if (flags & ZT_STORE_FINISH_OUTPUT) out.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_gaussian(const char* in_path, const char* out_path, int dtype_out,
                      const char* encoding_json, const float* sigma,
                      const int64_t* kernel_half_size, int device, int64_t row_begin,
                      int64_t row_end, int nthreads, int flags, zt_store_stats* stats) {
    try {
        if (!in_path || !out_path || !sigma || !kernel_half_size)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null argument");
        Array in = Array::open(in_path);
        const int nd = in.ndim();
        for (int d = 0; d < nd; ++d)
            if (kernel_half_size[d] < 0)
                return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "negative kernel_half_size");
        Array out = build_output(in, out_path, dtype_out, in.shape, encoding_json);
        const int dt = out.dtype;
        if (int rc = zt_gaussian_is_compatible(in.dtype, dt)) return rc;
        if (flags & ZT_STORE_ERASE_OUTPUT_METADATA) out.erase_metadata();
        const int64_t halo = kernel_half_size[0], nz = in.shape[0];
        RowOp op;
        op.input_planes = [&](int64_t z0, int64_t z1, int64_t& a, int64_t& b) {
            a = std::max<int64_t>(0, z0 - halo);  // ArraySubsetOverlap (gaussian.rs:86-87)
            b = std::min(nz, z1 + halo);
        };
        const std::vector<int64_t> shape = in.shape;
        const std::vector<float> sg(sigma, sigma + nd);
        const std::vector<int64_t> hs(kernel_half_size, kernel_half_size + nd);
        const int din = in.dtype;
        int64_t gplane = 1;
        for (int d = 1; d < nd; ++d) gplane *= shape[d];
        op.scratch_bytes = [&](int64_t planes) -> uint64_t {
            return (uint64_t)planes * gplane * 8;  // two f32 pass buffers
        };
        op.apply = [&](zt_ctx* c, const void* slab, int64_t in0, int64_t in1, void* o, int64_t z0,
                       int64_t z1) -> int {
            // the slab is a block that carries the halo or reaches the array edge on axis 0 and
            // spans the other axes: its result on [z0, z1) is the chunked result
            std::vector<int64_t> bshape(shape), ostart(nd, 0), oshape(shape);
            bshape[0] = in1 - in0;
            ostart[0] = z0 - in0;
            oshape[0] = z1 - z0;
            return zt_gaussian_apply_ndarray(c, din, slab, bshape.data(), nd, ostart.data(),
                                             oshape.data(), dt, o, sg.data(), hs.data());
        };
        run_pipeline(in, out, device, row_begin, row_end, nthreads, op, stats);
        if (flags & ZT_STORE_FINISH_OUTPUT) out.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

int zt_store_downsample_gaussian(const char* in_path, const char* out_path, const int64_t* stride,
                                 const float* sigma, const int64_t* kernel_half_size,
                                 int dtype_out, const char* encoding_json, int device,
                                 int64_t row_begin, int64_t row_end, int nthreads, int flags,
                                 zt_store_stats* stats) {
    try {
        if (!in_path || !out_path || !stride || !sigma || !kernel_half_size)
            return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "null argument");
        Array in = Array::open(in_path);
        const int nd = in.ndim();
        for (int d = 0; d < nd; ++d)
            if (kernel_half_size[d] < 0)
                return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "negative kernel_half_size");
        std::vector<int64_t> st(stride, stride + nd), oshape(nd), win(nd);
        if (int rc = zt_downsample_output_shape(in.shape.data(), nd, st.data(), oshape.data()))
            return rc;
        for (int d = 0; d < nd; ++d) win[d] = std::min(st[d], in.shape[d]);
        Array out = build_output(in, out_path, dtype_out, oshape, encoding_json);
        const int dt = out.dtype;
        if (int rc = zt_downsample_is_compatible(zt::kF32, dt, 0)) return rc;
        if (flags & ZT_STORE_ERASE_OUTPUT_METADATA) out.erase_metadata();
        const int64_t w0 = win[0], halo = kernel_half_size[0], nz = in.shape[0];
        auto ds_planes = [&](int64_t z0, int64_t z1, int64_t& a, int64_t& b) {
            a = z0 * w0;  // Downsample::input_subset (downsample.rs:64-70)
            b = std::min(z1 * w0, nz);
        };
        RowOp op;
        op.input_planes = [&](int64_t z0, int64_t z1, int64_t& a, int64_t& b) {
            ds_planes(z0, z1, a, b);  // plus the Gaussian halo (zarrs_ome.rs:251-255)
            a = std::max<int64_t>(0, a - halo);
            b = std::min(nz, b + halo);
        };
        const std::vector<int64_t> ishape = in.shape;
        const std::vector<float> sg(sigma, sigma + nd);
        const std::vector<int64_t> hs(kernel_half_size, kernel_half_size + nd);
        int64_t plane = 1;
        for (int d = 1; d < nd; ++d) plane *= ishape[d];
        DevBuf gtmp;  // the Gaussian of one row's downsample input (f32)
        const int din = in.dtype;
        op.apply = [&](zt_ctx* c, const void* slab, int64_t in0, int64_t in1, void* o, int64_t z0,
                       int64_t z1) -> int {
            int64_t a, b;
            ds_planes(z0, z1, a, b);
            if (!gtmp.p) gtmp.alloc(sizeof(float) * (size_t)(w0 * out.chunk_shape[0] * plane));
            std::vector<int64_t> bshape(ishape), gstart(nd, 0), gshape(ishape);
            bshape[0] = in1 - in0;
            gstart[0] = a - in0;
            gshape[0] = b - a;
            if (int rc = zt_gaussian_apply_ndarray(c, din, slab, bshape.data(), nd, gstart.data(),
                                                   gshape.data(), zt::kF32, gtmp.p, sg.data(),
                                                   hs.data()))
                return rc;
            return zt_downsample_apply_ndarray(c, zt::kF32, gtmp.p, gshape.data(), nd, st.data(),
                                               0, dt, o);
        };
        run_pipeline(in, out, device, row_begin, row_end, nthreads, op, stats);
        if (flags & ZT_STORE_FINISH_OUTPUT) out.store_metadata();
        return ZT_OK;
    } catch (const std::exception& e) {
        return report(e);
    }
}

void zt_store_set_progress_callback(zt_progress_fn fn, void* user) {
    std::lock_guard<std::mutex> lk(g_progress_mu);
    g_progress_fn = fn;
    g_progress_user = user;
}

int zt_store_set_chunk_limit(int64_t max_chunks) {
    if (max_chunks < 0) return zt::set_last_error(ZT_ERR_INVALID_PARAMETERS, "chunk limit must be >= 0");
    g_chunk_limit = max_chunks;
    return ZT_OK;
}

uint64_t zt_store_host_available_bytes(void) { return host_available_bytes(); }

int zt_store_codec_available(const char* name) {
    if (!name) return 0;
    std::string n(name);
    if (n == "bytes" || n == "gzip" || n == "crc32c" || n == "sharding_indexed") return 1;
    if (n == "zstd") return zt::zarr::zstd_available() ? 1 : 0;
    return 0;
}

}  // extern "C"
