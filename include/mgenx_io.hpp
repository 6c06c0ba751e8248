// mgenx_io.hpp -- batched UDP socket I/O for the mgenx batch path (header-only, C++17, Linux).
//
// The reference receives one datagram per RecvFrom call and sends one per SendTo
// (MgenUdpTransport::OnEvent, src/common/mgenTransport.cpp:938-997; SendMessage :1011-1063,
// SendPendingMessage :210-301).  Here the same socket work is done a batch at a time:
//   UdpTransport::Send   sendmmsg of n packed datagrams held in fixed slots of a slab
//                        (the layout SendBatch::Pack / mgenx_pack_batch produces);
//   UdpTransport::Recv   recvmmsg into fixed slots (the recvmmsg layout mgenx_unpack_batch
//                        reads with stride = slot), plus per-datagram length, source address
//                        (recvfrom's srcAddr, mgenTransport.cpp:947-957) and receive time
//                        (ProtoSystemTime after the receive, :953-954).
// Plain sockets: no HIP here; the slabs may be pinned host memory (PinnedArray) so the
// H2D copy that follows runs at full PCIe rate.
#pragma once

#include <arpa/inet.h>
#include <errno.h>
#include <netinet/in.h>
#include <sys/types.h>
#include <poll.h>
#include <sys/socket.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "mgenx.h"

namespace mgenx {

class UdpTransport {
 public:
  // bind to addr:port (port 0 = ephemeral); non-blocking.  addr is IPv4 ("127.0.0.1") or
  // IPv6 ("::1"): the socket family follows it, as ProtoSocket's does for its address.
  explicit UdpTransport(const char* addr = "127.0.0.1", uint16_t port = 0, int rcvbuf = 4 << 20) {
    memset(&local_, 0, sizeof(local_));
    sockaddr_in a4;
    sockaddr_in6 a6;
    memset(&a4, 0, sizeof(a4));
    memset(&a6, 0, sizeof(a6));
    socklen_t alen;
    if (inet_pton(AF_INET, addr, &a4.sin_addr) == 1) {
      a4.sin_family = AF_INET;
      a4.sin_port = htons(port);
      memcpy(&local_, &a4, sizeof(a4));
      alen = sizeof(a4);
    } else if (inet_pton(AF_INET6, addr, &a6.sin6_addr) == 1) {
      a6.sin6_family = AF_INET6;
      a6.sin6_port = htons(port);
      memcpy(&local_, &a6, sizeof(a6));
      alen = sizeof(a6);
    } else {
      throw std::runtime_error("bad address");
    }
    fd_ = ::socket(local_.ss_family, SOCK_DGRAM | SOCK_NONBLOCK, 0);
    if (fd_ < 0) throw std::runtime_error(std::string("socket: ") + strerror(errno));
    (void)::setsockopt(fd_, SOL_SOCKET, SO_RCVBUF, &rcvbuf, sizeof(rcvbuf));
    if (::bind(fd_, (sockaddr*)&local_, alen) != 0)
      throw std::runtime_error(std::string("bind: ") + strerror(errno));
    socklen_t l = sizeof(local_);
    ::getsockname(fd_, (sockaddr*)&local_, &l);
  }
  ~UdpTransport() {
    if (fd_ >= 0) ::close(fd_);
  }
  UdpTransport(const UdpTransport&) = delete;
  UdpTransport& operator=(const UdpTransport&) = delete;
  uint16_t Port() const {
    return local_.ss_family == AF_INET6 ? ntohs(((const sockaddr_in6&)local_).sin6_port)
                                        : ntohs(((const sockaddr_in&)local_).sin_port);
  }
  const sockaddr_storage& Local() const { return local_; }
  int Family() const { return local_.ss_family; }
  int fd() const { return fd_; }

  // sendmmsg datagram i = base[i * slot .. + lens[i]) to dst; zero-length entries (Pack
  // returned 0: MSG_SEND_FAILED) are skipped, as the reference does not send them.
  // Returns the number of datagrams the kernel accepted.
  uint32_t Send(const sockaddr_storage& dst, const uint8_t* base, uint32_t slot,
                const uint32_t* lens, uint32_t n) {
    const socklen_t dlen = dst.ss_family == AF_INET6 ? sizeof(sockaddr_in6) : sizeof(sockaddr_in);
    std::vector<mmsghdr> m;
    std::vector<iovec> iov;
    m.reserve(n);
    iov.reserve(n);
    for (uint32_t i = 0; i < n; i++) {
      if (!lens[i]) continue;
      iov.push_back({(void*)(base + (size_t)i * slot), lens[i]});
    }
    for (size_t i = 0; i < iov.size(); i++) {
      mmsghdr h;
      memset(&h, 0, sizeof(h));
      h.msg_hdr.msg_name = (void*)&dst;
      h.msg_hdr.msg_namelen = dlen;
      h.msg_hdr.msg_iov = &iov[i];
      h.msg_hdr.msg_iovlen = 1;
      m.push_back(h);
    }
    // A full socket buffer waits for POLLOUT (bounded); a datagram the kernel refuses
    // (e.g. EMSGSIZE) is skipped rather than dropping the rest of the batch.
    size_t done = 0, sent = 0;
    while (done < m.size()) {
      const int r = ::sendmmsg(fd_, m.data() + done, (unsigned)(m.size() - done), 0);
      if (r < 0) {
        if (errno == EINTR) continue;
        if (errno == EAGAIN || errno == EWOULDBLOCK) {
          pollfd p = {fd_, POLLOUT, 0};
          if (::poll(&p, 1, 1000) > 0) continue;
        }
        done += 1;  // hard error (or no progress for 1 s): skip this datagram
        continue;
      }
      done += (size_t)r;
      sent += (size_t)r;
    }
    return (uint32_t)sent;
  }

  // recvmmsg up to cap datagrams (non-blocking) into base[i * slot], i = 0..; per datagram:
  // length, source (mgenx_addr) and receive time.  Returns the number received (0 = none).
  uint32_t Recv(uint8_t* base, uint32_t slot, uint32_t cap, uint32_t* lens, mgenx_addr* src,
                uint32_t* rx_sec, uint32_t* rx_usec) {
    if (cap == 0) return 0;
    std::vector<mmsghdr> m(cap);
    std::vector<iovec> iov(cap);
    std::vector<sockaddr_storage> from(cap);
    for (uint32_t i = 0; i < cap; i++) {
      iov[i] = {base + (size_t)i * slot, slot};
      memset(&m[i], 0, sizeof(m[i]));
      m[i].msg_hdr.msg_name = &from[i];
      m[i].msg_hdr.msg_namelen = sizeof(from[i]);
      m[i].msg_hdr.msg_iov = &iov[i];
      m[i].msg_hdr.msg_iovlen = 1;
    }
    const int r = ::recvmmsg(fd_, m.data(), cap, MSG_DONTWAIT, nullptr);
    if (r <= 0) return 0;
    struct timeval now;
    gettimeofday(&now, nullptr);  // ProtoSystemTime after the receive
    for (int i = 0; i < r; i++) {
      lens[i] = m[i].msg_len;
      if (src) {  // recvfrom's source as a ProtoAddress (IPv4 or IPv6)
        memset(&src[i], 0, sizeof(src[i]));
        if (from[i].ss_family == AF_INET6) {
          const sockaddr_in6& f6 = (const sockaddr_in6&)from[i];
          src[i].type = 2;
          src[i].len = 16;
          src[i].port = ntohs(f6.sin6_port);
          memcpy(src[i].addr, &f6.sin6_addr, 16);
        } else {
          const sockaddr_in& f4 = (const sockaddr_in&)from[i];
          src[i].type = 1;
          src[i].len = 4;
          src[i].port = ntohs(f4.sin_port);
          memcpy(src[i].addr, &f4.sin_addr, 4);
        }
      }
      if (rx_sec) rx_sec[i] = (uint32_t)now.tv_sec;
      if (rx_usec) rx_usec[i] = (uint32_t)now.tv_usec;
    }
    return (uint32_t)r;
  }

 private:
  int fd_ = -1;
  sockaddr_storage local_{};
};

}  // namespace mgenx
