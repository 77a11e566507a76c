// zt_zarr.hpp — Zarr V3 filesystem arrays for the store -> store filter path.
//
// What the reference gets from zarrs 0.20.0-beta.2 (Cargo.lock) on this path: array metadata
// (zarr.json), the regular chunk grid, chunk key encodings, fill values and the codec chain
// (`bytes`, `gzip`, `zstd`, `crc32c`, `sharding_indexed`), used through
// Array::retrieve_array_subset_ndarray / store_array_subset_ndarray in apply_chunk
// (guided_filter.rs:95-110) and zarrs_ome's level loop (zarrs_ome.rs:226-232). Restated here from
// the Zarr V3 specification; chunks are decoded into / encoded from strided host regions so a
// whole chunk row can be assembled once and shared by every halo that reads it.
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "zt_json.hpp"

namespace zt {
namespace zarr {

// Raised for storage / metadata / codec problems; `code` is a zt_status value.
struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

int dtype_from_name(const std::string& name);   // zt_dtype, or -1

// Metadata of an array that is not finished yet (written by several processes); Array::open
// falls back to it when zarr.json is absent.
constexpr const char* kPendingMetadata = ".zt_pending.json";
const char* dtype_name(int dtype);
size_t dtype_size(int dtype);

// One bytes -> bytes codec (gzip, zstd, crc32c).
struct BytesCodec {
    std::string name;
    int level = 0;
    bool checksum = false;
    std::vector<uint8_t> encode(const std::vector<uint8_t>& in) const;
    std::vector<uint8_t> decode(const std::vector<uint8_t>& in, size_t expect) const;
    json::Value to_json() const;
};

// A codec chain: [bytes | sharding_indexed] followed by bytes -> bytes codecs.
struct CodecChain {
    bool big_endian = false;
    std::vector<BytesCodec> b2b;
    // sharding_indexed (when `sharded`): inner chunk shape, inner chain, index chain
    bool sharded = false;
    std::vector<int64_t> inner_shape;
    std::shared_ptr<CodecChain> inner, index;
    bool index_at_end = true;

    static CodecChain from_json(const json::Value& codecs, int ndim);
    json::Value to_json() const;
    // Encode / decode one chunk of `shape` (C order, `esz`-byte elements).
    std::vector<uint8_t> encode(const uint8_t* raw, const std::vector<int64_t>& shape, size_t esz,
                                const uint8_t* fill) const;
    // Decodes into `raw` (shape elements). Returns false if the chunk is absent in a shard.
    void decode(const std::vector<uint8_t>& bytes, uint8_t* raw,
                const std::vector<int64_t>& shape, size_t esz, const uint8_t* fill) const;
    std::vector<uint8_t> encode_bytes(std::vector<uint8_t> raw, size_t esz) const;
    std::vector<uint8_t> decode_bytes(const std::vector<uint8_t>& bytes, size_t raw_bytes,
                                      size_t esz) const;
};

class Array {
  public:
    std::string path;
    std::vector<int64_t> shape, chunk_shape;
    int dtype = -1;
    size_t esz = 0;
    std::vector<uint8_t> fill;  // one element
    json::Value fill_json;
    std::string key_encoding = "default";
    char separator = '/';
    CodecChain codecs;
    json::Value attributes, dimension_names;

    static Array open(const std::string& path);
    // A new array (zarr.json written by store_metadata()).
    static Array create(const std::string& path, int dtype, const std::vector<int64_t>& shape,
                        const std::vector<int64_t>& chunk_shape, const json::Value& codecs,
                        const json::Value& fill_value);
    json::Value metadata() const;
    void store_metadata() const;
    void erase_metadata() const;

    int ndim() const { return (int)shape.size(); }
    std::vector<int64_t> grid_shape() const;
    std::string chunk_key(const int64_t* idx) const;
    std::string chunk_path(const int64_t* idx) const { return path + "/" + chunk_key(idx); }
    int64_t chunk_elems() const;

    // Decode chunk `idx` into the region of a C-order host buffer whose element strides are
    // `dst_strides` and whose origin is at array coordinate `dst_origin`; only the part of the
    // chunk inside the array AND inside [dst_origin, dst_origin + dst_shape) is written. Missing
    // chunks read as the fill value. Returns the number of encoded bytes read from storage.
    size_t read_chunk(const int64_t* idx, uint8_t* dst, const int64_t* dst_origin,
                      const int64_t* dst_shape, const int64_t* dst_strides) const;
    // Encode chunk `idx` from the same kind of region (must cover the chunk's in-array part);
    // elements beyond the array edge are written as the fill value. Returns bytes written.
    size_t write_chunk(const int64_t* idx, const uint8_t* src, const int64_t* src_origin,
                       const int64_t* src_shape, const int64_t* src_strides) const;
};

// Fill-value JSON for a dtype from a double (NaN/Infinity as strings), and the element bytes of a
// fill-value JSON (Zarr V3 fill_value grammar: number, bool, "NaN", "Infinity", "-Infinity",
// "0x..." raw hex).
json::Value fill_json_from_double(int dtype, double v);
std::vector<uint8_t> fill_bytes(int dtype, const json::Value& v);

// Strided copy of an n-D box between two C-order buffers (element size esz).
void copy_box(const uint8_t* src, const int64_t* src_strides, uint8_t* dst,
              const int64_t* dst_strides, const int64_t* box, int ndim, size_t esz);

uint32_t crc32c(const uint8_t* p, size_t n);
bool zstd_available();

}  // namespace zarr
}  // namespace zt
