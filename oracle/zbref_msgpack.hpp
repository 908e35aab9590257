// ORACLE / TEST INFRASTRUCTURE ONLY. Never linked into the product (zeebe_amd/csrc).
//
// msgpack encoding/decoding restated from the reference:
//   writer: msgpack-core/src/main/java/io/zeebe/msgpack/spec/MsgPackWriter.java:94-305
//   reader: msgpack-core/src/main/java/io/zeebe/msgpack/spec/MsgPackReader.java:38-400
//   formats: msgpack-core/src/main/java/io/zeebe/msgpack/spec/MsgPackFormat.java
// All multi-byte values are big endian (MsgPackCodes.BYTE_ORDER).
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace zbref {

using bytes = std::string;

struct ZbError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---------------------------------------------------------------- writer
struct MpWriter {
  bytes b;
  void u8(uint8_t v) { b.push_back((char)v); }
  void be16(uint16_t v) { u8(v >> 8); u8(v & 0xff); }
  void be32(uint32_t v) { be16(v >> 16); be16(v & 0xffff); }
  void be64(uint64_t v) { be32((uint32_t)(v >> 32)); be32((uint32_t)v); }
  void raw(const bytes& s) { b += s; }
  void raw(const char* p, size_t n) { b.append(p, n); }
  // MsgPackWriter.writeMapHeader :58-77
  void map_header(uint32_t n) {
    if (n < 16) u8(0x80 | n);
    else if (n < 65536) { u8(0xde); be16((uint16_t)n); }
    else { u8(0xdf); be32(n); }
  }
  // writeArrayHeader :38-56
  void array_header(uint32_t n) {
    if (n < 16) u8(0x90 | n);
    else if (n < 65536) { u8(0xdc); be16((uint16_t)n); }
    else { u8(0xdd); be32(n); }
  }
  // writeStringHeader :202-222
  void str_header(uint32_t n) {
    if (n < 32) u8(0xa0 | n);
    else if (n < 256) { u8(0xd9); u8((uint8_t)n); }
    else if (n < 65536) { u8(0xda); be16((uint16_t)n); }
    else { u8(0xdb); be32(n); }
  }
  void str(const bytes& s) { str_header((uint32_t)s.size()); raw(s); }
  // writeBinaryHeader :231-250
  void bin(const bytes& s) {
    uint32_t n = (uint32_t)s.size();
    if (n < 256) { u8(0xc4); u8((uint8_t)n); }
    else if (n < 65536) { u8(0xc5); be16((uint16_t)n); }
    else { u8(0xc6); be32(n); }
    raw(s);
  }
  // writeInteger :143-201 (signed semantics)
  void integer(int64_t v) {
    if (v < -(1LL << 5)) {
      if (v < -(1LL << 15)) {
        if (v < -(1LL << 31)) { u8(0xd3); be64((uint64_t)v); }
        else { u8(0xd2); be32((uint32_t)(int32_t)v); }
      } else {
        if (v < -(1 << 7)) { u8(0xd1); be16((uint16_t)(int16_t)v); }
        else { u8(0xd0); u8((uint8_t)(int8_t)v); }
      }
    } else if (v < (1 << 7)) {
      u8((uint8_t)(int8_t)v);
    } else {
      if (v < (1LL << 16)) {
        if (v < (1 << 8)) { u8(0xcc); u8((uint8_t)v); }
        else { u8(0xcd); be16((uint16_t)v); }
      } else {
        if (v < (1LL << 32)) { u8(0xce); be32((uint32_t)v); }
        else { u8(0xcf); be64((uint64_t)v); }
      }
    }
  }
  void boolean(bool v) { u8(v ? 0xc3 : 0xc2); }
  void nil() { u8(0xc0); }
  // writeFloat :286-305: float32 iff exactly representable
  void floating(double v) {
    float f = (float)v;
    if ((double)f == v) {
      uint32_t u; std::memcpy(&u, &f, 4); u8(0xca); be32(u);
    } else {
      uint64_t u; std::memcpy(&u, &v, 8); u8(0xcb); be64(u);
    }
  }
};

// ---------------------------------------------------------------- reader / tokens
enum class MpType { INTEGER, FLOAT, BOOLEAN, NIL, MAP, ARRAY, BINARY, STRING, EXTENSION, NEVER_USED };

inline const char* mp_type_name(MpType t) {
  switch (t) {
    case MpType::INTEGER: return "INTEGER";
    case MpType::FLOAT: return "FLOAT";
    case MpType::BOOLEAN: return "BOOLEAN";
    case MpType::NIL: return "NIL";
    case MpType::MAP: return "MAP";
    case MpType::ARRAY: return "ARRAY";
    case MpType::BINARY: return "BINARY";
    case MpType::STRING: return "STRING";
    case MpType::EXTENSION: return "EXTENSION";
    default: return "NEVER_USED";
  }
}

inline bool mp_is_scalar(MpType t) { return t != MpType::MAP && t != MpType::ARRAY; }

// MsgPackFormat.valueOf -> type (MsgPackFormat.java)
inline MpType mp_format_type(uint8_t b) {
  if (b <= 0x7f) return MpType::INTEGER;
  if (b <= 0x8f) return MpType::MAP;
  if (b <= 0x9f) return MpType::ARRAY;
  if (b <= 0xbf) return MpType::STRING;
  if (b >= 0xe0) return MpType::INTEGER;
  switch (b) {
    case 0xc0: return MpType::NIL;
    case 0xc1: return MpType::NEVER_USED;
    case 0xc2: case 0xc3: return MpType::BOOLEAN;
    case 0xc4: case 0xc5: case 0xc6: return MpType::BINARY;
    case 0xc7: case 0xc8: case 0xc9: return MpType::EXTENSION;
    case 0xca: case 0xcb: return MpType::FLOAT;
    case 0xcc: case 0xcd: case 0xce: case 0xcf:
    case 0xd0: case 0xd1: case 0xd2: case 0xd3: return MpType::INTEGER;
    case 0xd4: case 0xd5: case 0xd6: case 0xd7: case 0xd8: return MpType::EXTENSION;
    case 0xd9: case 0xda: case 0xdb: return MpType::STRING;
    case 0xdc: case 0xdd: return MpType::ARRAY;
    case 0xde: case 0xdf: return MpType::MAP;
  }
  return MpType::NEVER_USED;
}

struct MpToken {
  MpType type = MpType::NIL;
  int64_t ival = 0;
  double fval = 0;
  bool bval = false;
  uint32_t size = 0;            // map: #entries, array: #elements
  const uint8_t* data = nullptr;  // string/binary payload
  uint32_t len = 0;
  uint32_t total = 0;           // encoded length of the token header (+payload for str/bin)
  bytes value() const { return bytes((const char*)data, len); }
};

struct MpReader {
  const uint8_t* buf;
  size_t cap;
  size_t off = 0;
  MpReader(const uint8_t* p, size_t n) : buf(p), cap(n) {}
  explicit MpReader(const bytes& s) : buf((const uint8_t*)s.data()), cap(s.size()) {}
  uint8_t byte_at(size_t o) const {
    if (o >= cap) throw ZbError("Index out of bounds");
    return buf[o];
  }
  uint16_t be16(size_t o) const { return (uint16_t)((byte_at(o) << 8) | byte_at(o + 1)); }
  uint32_t be32(size_t o) const { return ((uint32_t)be16(o) << 16) | be16(o + 2); }
  uint64_t be64(size_t o) const { return ((uint64_t)be32(o) << 32) | be32(o + 4); }
  bool has_next() const { return off < cap; }

  uint32_t read_map_header() {
    uint8_t h = byte_at(off++);
    if ((h & 0xf0) == 0x80) return h & 0x0f;
    if (h == 0xde) { uint32_t n = be16(off); off += 2; return n; }
    if (h == 0xdf) { int32_t n = (int32_t)be32(off); off += 4; if (n < 0) throw ZbError("negative"); return (uint32_t)n; }
    throw ZbError("Unable to determine map type");
  }
  uint32_t read_array_header() {
    uint8_t h = byte_at(off++);
    if ((h & 0xf0) == 0x90) return h & 0x0f;
    if (h == 0xdc) { uint32_t n = be16(off); off += 2; return n; }
    if (h == 0xdd) { int32_t n = (int32_t)be32(off); off += 4; if (n < 0) throw ZbError("negative"); return (uint32_t)n; }
    throw ZbError("Unable to determine array type");
  }
  uint32_t read_string_length() {
    uint8_t h = byte_at(off++);
    if ((h & 0xe0) == 0xa0) return h & 0x1f;
    if (h == 0xd9) { return byte_at(off++); }
    if (h == 0xda) { uint32_t n = be16(off); off += 2; return n; }
    if (h == 0xdb) { int32_t n = (int32_t)be32(off); off += 4; if (n < 0) throw ZbError("negative"); return (uint32_t)n; }
    throw ZbError("Unable to determine string type");
  }
  uint32_t read_binary_length() {
    uint8_t h = byte_at(off++);
    if (h == 0xc4) return byte_at(off++);
    if (h == 0xc5) { uint32_t n = be16(off); off += 2; return n; }
    if (h == 0xc6) { int32_t n = (int32_t)be32(off); off += 4; if (n < 0) throw ZbError("negative"); return (uint32_t)n; }
    throw ZbError("Unable to determine binary type");
  }
  int64_t read_integer() {
    uint8_t h = byte_at(off++);
    if (h <= 0x7f || h >= 0xe0) return (int8_t)h;
    switch (h) {
      case 0xcc: return byte_at(off++);
      case 0xcd: { int64_t v = be16(off); off += 2; return v; }
      case 0xce: { int64_t v = be32(off); off += 4; return v; }
      case 0xcf: { int64_t v = (int64_t)be64(off); off += 8; if (v < 0) throw ZbError("negative"); return v; }
      case 0xd0: return (int8_t)byte_at(off++);
      case 0xd1: { int64_t v = (int16_t)be16(off); off += 2; return v; }
      case 0xd2: { int64_t v = (int32_t)be32(off); off += 4; return v; }
      case 0xd3: { int64_t v = (int64_t)be64(off); off += 8; return v; }
    }
    throw ZbError("Unable to determine long type");
  }
  double read_float() {
    uint8_t h = byte_at(off++);
    if (h == 0xca) { uint32_t u = be32(off); off += 4; float f; std::memcpy(&f, &u, 4); return f; }
    if (h == 0xcb) { uint64_t u = be64(off); off += 8; double d; std::memcpy(&d, &u, 8); return d; }
    throw ZbError("Unable to determine float type");
  }
  // readToken :302-345
  MpToken read_token() {
    MpToken t;
    uint8_t b = byte_at(off);
    size_t start = off;
    MpType ty = mp_format_type(b);
    switch (ty) {
      case MpType::INTEGER: t.type = ty; t.ival = read_integer(); break;
      case MpType::FLOAT: t.type = ty; t.fval = read_float(); break;
      case MpType::BOOLEAN: t.type = ty; t.bval = byte_at(off++) == 0xc3; break;
      case MpType::MAP: t.type = ty; t.size = read_map_header(); break;
      case MpType::ARRAY: t.type = ty; t.size = read_array_header(); break;
      case MpType::NIL: t.type = ty; off++; break;
      case MpType::BINARY: {
        t.type = ty; uint32_t n = read_binary_length();
        if (off + n > cap) throw ZbError("Index out of bounds");
        t.data = buf + off; t.len = n; off += n; break;
      }
      case MpType::STRING: {
        t.type = ty; uint32_t n = read_string_length();
        if (off + n > cap) throw ZbError("Index out of bounds");
        t.data = buf + off; t.len = n; off += n; break;
      }
      default: throw ZbError("Unsupported token format");
    }
    t.total = (uint32_t)(off - start);
    return t;
  }
  // skipValues :347-438
  void skip_values(int64_t count) {
    while (count > 0) {
      uint8_t b = byte_at(off++);
      if (b <= 0x7f || b >= 0xe0 || b == 0xc0 || b == 0xc2 || b == 0xc3) {
      } else if ((b & 0xf0) == 0x80) count += (int64_t)(b & 0x0f) * 2;
      else if ((b & 0xf0) == 0x90) count += (b & 0x0f);
      else if ((b & 0xe0) == 0xa0) off += (b & 0x1f);
      else switch (b) {
        case 0xd0: case 0xcc: off += 1; break;
        case 0xd1: case 0xcd: off += 2; break;
        case 0xd2: case 0xce: case 0xca: off += 4; break;
        case 0xd3: case 0xcf: case 0xcb: off += 8; break;
        case 0xc4: case 0xd9: off += 1 + byte_at(off); break;
        case 0xc5: case 0xda: off += 2 + be16(off); break;
        case 0xc6: case 0xdb: off += 4 + be32(off); break;
        case 0xd4: off += 2; break;
        case 0xd5: off += 3; break;
        case 0xd6: off += 5; break;
        case 0xd7: off += 9; break;
        case 0xd8: off += 17; break;
        case 0xc7: off += 1 + 1 + byte_at(off); break;
        case 0xc8: off += 1 + 2 + be16(off); break;
        case 0xc9: off += 1 + 4 + be32(off); break;
        case 0xdc: count += be16(off); off += 2; break;
        case 0xdd: count += be32(off); off += 4; break;
        case 0xde: count += (int64_t)be16(off) * 2; off += 2; break;
        case 0xdf: count += (int64_t)be32(off) * 2; off += 4; break;
        default: throw ZbError("Encountered 0xC1 \"NEVER_USED\" byte");
      }
      count--;
    }
  }
};

}  // namespace zbref
