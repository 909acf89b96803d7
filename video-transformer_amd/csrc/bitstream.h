// bitstream.h — H.264 RBSP bit writer/reader and NAL emulation prevention
// (ITU-T H.264 §7.2 ue(v)/se(v)/u(n), §7.4.1 emulation_prevention_three_byte).
// Host side only: the synthetic stream writer and SPS/PPS parsing.
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace vts {

class BitWriter {
 public:
  void u(int n, uint32_t v) {
    for (int i = n - 1; i >= 0; --i) bit((v >> i) & 1u);
  }
  void bit(uint32_t b) {
    cur_ = static_cast<uint8_t>((cur_ << 1) | (b & 1u));
    if (++nbits_ == 8) {
      buf_.push_back(cur_);
      cur_ = 0;
      nbits_ = 0;
    }
  }
  void ue(uint32_t v) {  // Exp-Golomb, §9.1
    const uint64_t x = static_cast<uint64_t>(v) + 1;
    int len = 0;
    while ((x >> len) > 1) ++len;
    for (int i = 0; i < len; ++i) bit(0);
    for (int i = len; i >= 0; --i) bit(static_cast<uint32_t>((x >> i) & 1u));
  }
  void se(int32_t v) {  // §9.1.1
    ue(v > 0 ? static_cast<uint32_t>(2 * v - 1) : static_cast<uint32_t>(-2 * static_cast<int64_t>(v)));
  }
  bool aligned() const { return nbits_ == 0; }
  void align_zero() {
    while (nbits_ != 0) bit(0);
  }
  void trailing() {  // rbsp_trailing_bits()
    bit(1);
    align_zero();
  }
  void bytes(const uint8_t *p, size_t n) {  // byte-aligned raw bytes
    buf_.insert(buf_.end(), p, p + n);
  }
  std::vector<uint8_t> &data() { return buf_; }

 private:
  std::vector<uint8_t> buf_;
  uint8_t cur_ = 0;
  int nbits_ = 0;
};

// RBSP -> NAL payload bytes with emulation_prevention_three_byte inserted.
inline void append_ebsp(std::vector<uint8_t> &out, const uint8_t *rbsp, size_t n) {
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t b = rbsp[i];
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(b);
    zeros = (b == 0) ? zeros + 1 : 0;
  }
  // A trailing zero byte at the end of the NAL would need cabac_zero_word
  // handling; rbsp_trailing_bits guarantees the last byte is non-zero.
}

class BitReader {  // reads an EBSP (NAL payload) skipping emulation bytes
 public:
  BitReader(const uint8_t *p, size_t n) : p_(p), n_(n) {}
  bool ok() const { return !err_; }
  // 7.2 more_rbsp_data(): a bit other than the rbsp_stop_one_bit remains
  // (positions in EBSP bits; an emulation byte cannot follow the stop bit)
  bool more_rbsp_data() const {
    size_t last = n_;
    while (last > 0 && p_[last - 1] == 0) --last;
    if (last == 0) return false;
    int tz = 0;
    while (!((p_[last - 1] >> tz) & 1)) ++tz;
    const size_t stop = (last - 1) * 8 + static_cast<size_t>(7 - tz);
    return pos_ * 8 - static_cast<size_t>(bitpos_) < stop;
  }
  uint32_t bit() {
    if (bitpos_ == 0) {
      if (pos_ >= n_) {
        err_ = true;
        return 0;
      }
      if (zeros_ >= 2 && p_[pos_] == 3) {  // emulation prevention byte
        ++pos_;
        zeros_ = 0;
        if (pos_ >= n_) {
          err_ = true;
          return 0;
        }
      }
      byte_ = p_[pos_++];
      zeros_ = (byte_ == 0) ? zeros_ + 1 : 0;
      bitpos_ = 8;
    }
    --bitpos_;
    return (byte_ >> bitpos_) & 1u;
  }
  uint32_t u(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | bit();
    return v;
  }
  uint32_t ue() {
    int lz = 0;
    while (bit() == 0) {
      if (++lz > 31 || err_) {
        err_ = true;
        return 0;
      }
    }
    if (lz == 0) return 0;
    return static_cast<uint32_t>((1ull << lz) - 1 + u(lz));
  }
  int32_t se() {
    const uint32_t k = ue();
    return (k & 1u) ? static_cast<int32_t>((k + 1) / 2) : -static_cast<int32_t>(k / 2);
  }

 private:
  const uint8_t *p_;
  size_t n_;
  size_t pos_ = 0;
  int bitpos_ = 0;
  uint8_t byte_ = 0;
  int zeros_ = 0;
  bool err_ = false;
};

}  // namespace vts
