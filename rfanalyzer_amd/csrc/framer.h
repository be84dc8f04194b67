// Host-side frame assembly of Scheduler.run's FFT branch (no HIP; shared by
// librfa's rfa_push_packet and the sanitizer driver tests/sanitize/san_driver.cpp).
//
// Reference: Scheduler.kt:252-273 keeps one SamplePacket(fftSize) and fills it
// packet after packet through the converter's fillPacketIntoSamplePacket
// (Signed8BitIQConverter.java:80-98, Unsigned8BitIQConverter.java:80-98,
// Signed16BitIQConverter.kt:89-124): each packet's samples go in from the packet
// start at startIndex = samplePacket.size() until the buffer is full; the rest
// of that packet is dropped; frequency / sampleRate of the buffer are those of
// the last packet that filled it.  So a packet of P samples gives one frame per
// packet when P >= N, and one frame every ceil(N / P) packets when P < N.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <vector>

namespace rfa {

class PacketFramer {
public:
    // frame of n samples of bps bytes each; an empty partial frame
    void configure(size_t n, size_t bps) {
        n_ = n;
        bps_ = bps;
        buf_.assign(n * bps, 0);
        filled_ = 0;
    }
    // Copy the packet's leading whole samples into the partial frame.  Returns
    // true when the frame is now complete (its bytes: data(); call clear() once
    // it has been consumed).  Trailing bytes of a sample that is cut off by the
    // end of the packet are ignored (the JVM loop would index past the array).
    bool push(const void *packet, size_t bytes) {
        if (!n_ || filled_ >= n_) return filled_ >= n_ && n_ > 0;
        const size_t have = bytes / bps_;
        const size_t take = have < n_ - filled_ ? have : n_ - filled_;
        if (take) std::memcpy(buf_.data() + filled_ * bps_, packet, take * bps_);
        filled_ += take;
        return filled_ == n_;
    }
    void clear() { filled_ = 0; }
    const uint8_t *data() const { return buf_.data(); }
    size_t filled() const { return filled_; }  // samples in the partial frame
    size_t size() const { return n_; }

private:
    std::vector<uint8_t> buf_;
    size_t n_ = 0, bps_ = 0, filled_ = 0;
};

}  // namespace rfa
