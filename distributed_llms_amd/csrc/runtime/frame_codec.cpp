// Control-plane wire-frame codec.
//
// Replaces the reference's "10 ASCII bytes of pickle-header length + pickle(header)
// + raw payload" framing (src/network/protocol.py:38-129), which unpickles
// attacker-controlled bytes and reassembles payloads in O(n^2) 4 KiB chunks
// (SURVEY §2.9 D18).  Frame layout (little endian, 24-byte fixed prefix):
//
//   0  u32 magic   'DLLM' (0x4D4C4C44)
//   4  u8  version (1)
//   5  u8  flags
//   6  u16 command id (index into the protocol's command table)
//   8  u32 header length  (UTF-8 JSON object)
//  12  u64 payload length (raw bytes: token ids, tensors, shard files)
//  20  u32 CRC-32 of the header bytes
//
// The payload is streamed with recv_into() into one preallocated buffer.
#include <pybind11/pybind11.h>

#include <array>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

constexpr uint32_t kMagic = 0x4D4C4C44u;  // "DLLM" little-endian
constexpr uint8_t kVersion = 1;
constexpr size_t kPrefix = 24;
constexpr uint32_t kMaxHeader = 16u << 20;         // 16 MiB of JSON is already absurd
constexpr uint64_t kMaxPayload = 1ull << 40;        // 1 TiB sanity bound

std::array<uint32_t, 256> make_crc_table() {
  std::array<uint32_t, 256> t{};
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    t[i] = c;
  }
  return t;
}

uint32_t crc32(const uint8_t* p, size_t n) {
  static const auto table = make_crc_table();
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return c ^ 0xFFFFFFFFu;
}

template <typename T>
void put(uint8_t* dst, T v) {
  std::memcpy(dst, &v, sizeof(T));
}
template <typename T>
T get(const uint8_t* src) {
  T v;
  std::memcpy(&v, src, sizeof(T));
  return v;
}

}  // namespace

// -> prefix (24 bytes) + header bytes, ready for sendall(); payload is sent separately.
py::bytes encode_frame_head(int command_id, int flags, py::bytes header, uint64_t payload_len) {
  std::string h = header;
  if (command_id < 0 || command_id > 0xFFFF) throw std::invalid_argument("command id out of range");
  if (h.size() > kMaxHeader) throw std::invalid_argument("header too large");
  if (payload_len > kMaxPayload) throw std::invalid_argument("payload too large");
  std::string out(kPrefix + h.size(), '\0');
  auto* p = reinterpret_cast<uint8_t*>(&out[0]);
  put<uint32_t>(p + 0, kMagic);
  put<uint8_t>(p + 4, kVersion);
  put<uint8_t>(p + 5, (uint8_t)flags);
  put<uint16_t>(p + 6, (uint16_t)command_id);
  put<uint32_t>(p + 8, (uint32_t)h.size());
  put<uint64_t>(p + 12, payload_len);
  put<uint32_t>(p + 20, crc32(reinterpret_cast<const uint8_t*>(h.data()), h.size()));
  std::memcpy(p + kPrefix, h.data(), h.size());
  return py::bytes(out);
}

// prefix (24 bytes) -> (command_id, flags, header_len, payload_len, header_crc)
py::tuple decode_frame_prefix(py::bytes prefix) {
  std::string s = prefix;
  if (s.size() != kPrefix) throw std::invalid_argument("frame prefix must be 24 bytes");
  auto* p = reinterpret_cast<const uint8_t*>(s.data());
  if (get<uint32_t>(p) != kMagic) throw std::invalid_argument("bad frame magic");
  if (get<uint8_t>(p + 4) != kVersion) throw std::invalid_argument("unsupported frame version");
  const uint32_t hl = get<uint32_t>(p + 8);
  const uint64_t pl = get<uint64_t>(p + 12);
  if (hl > kMaxHeader) throw std::invalid_argument("header length out of bounds");
  if (pl > kMaxPayload) throw std::invalid_argument("payload length out of bounds");
  return py::make_tuple((int)get<uint16_t>(p + 6), (int)get<uint8_t>(p + 5), hl, pl, get<uint32_t>(p + 20));
}

bool check_header_crc(py::bytes header, uint32_t expected) {
  std::string h = header;
  return crc32(reinterpret_cast<const uint8_t*>(h.data()), h.size()) == expected;
}

uint32_t crc32_bytes(py::bytes b) {
  std::string h = b;
  return crc32(reinterpret_cast<const uint8_t*>(h.data()), h.size());
}

void register_frame_codec(py::module_& m) {
  m.attr("FRAME_PREFIX_SIZE") = (int)kPrefix;
  m.attr("FRAME_MAGIC") = kMagic;
  m.def("encode_frame_head", &encode_frame_head, py::arg("command_id"), py::arg("flags"), py::arg("header"),
        py::arg("payload_len"));
  m.def("decode_frame_prefix", &decode_frame_prefix);
  m.def("check_header_crc", &check_header_crc);
  m.def("crc32", &crc32_bytes);
}
