// Core of the shared-memory request/response channel (no Python): segment layout, sequence protocol,
// futex waits.  Used by the pybind11 module (shm_channel.cpp) and the native TSan stress test
// (tests/native/shm_stress.cpp).  See shm_channel.cpp for the protocol description.
#pragma once
#include <atomic>
#include <cerrno>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstring>
#include <fcntl.h>
#include <linux/futex.h>
#include <signal.h>
#include <stdexcept>
#include <string>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>
#include <vector>

namespace as_host {

constexpr uint64_t kMagic = 0x4153544d43484e31ull;  // "ASTMCHN1"
constexpr size_t kPage = 4096;

struct alignas(64) Header {
  uint64_t magic;
  uint32_t n_slots;
  uint32_t _pad0;
  uint64_t slot_bytes;
  std::atomic<uint32_t> doorbell;  // bumped on every request: the server's futex word
  std::atomic<uint32_t> closed;
};

struct alignas(64) Slot {
  std::atomic<uint32_t> req_seq;   // written by the client
  std::atomic<uint32_t> resp_seq;  // written by the server
  std::atomic<uint64_t> req_len;
  std::atomic<uint64_t> resp_len;
  std::atomic<int32_t> pid;        // client pid (0 = free)
  std::atomic<uint32_t> tag;       // free-form client tag (player / kind routing)
};

static_assert(std::atomic<uint32_t>::is_always_lock_free, "futex words must be lock free");
static_assert(std::atomic<uint64_t>::is_always_lock_free, "64-bit atomics must be lock free");

size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

long futex_wait(std::atomic<uint32_t>* addr, uint32_t expected, int timeout_ms) {
  timespec ts{}, *pts = nullptr;
  if (timeout_ms >= 0) {
    ts.tv_sec = timeout_ms / 1000;
    ts.tv_nsec = static_cast<long>(timeout_ms % 1000) * 1000000L;
    pts = &ts;
  }
  // shared (non-private) futex: the word lives in memory mapped by several processes
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, expected, pts, nullptr, 0);
}

void futex_wake(std::atomic<uint32_t>* addr, int n) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAKE, n, nullptr, nullptr, 0);
}

int64_t now_ms() {
  return std::chrono::duration_cast<std::chrono::milliseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

class Segment {
 public:
  Segment(const std::string& name, uint32_t n_slots, uint64_t slot_bytes, bool create) : name_(name), owner_(create) {
    if (create) {
      if (n_slots == 0 || slot_bytes == 0) throw std::invalid_argument("n_slots and slot_bytes must be > 0");
      slot_bytes = round_up(slot_bytes, kPage);
      size_ = layout_size(n_slots, slot_bytes);
      int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(create) failed for " + name + ": " + strerror(errno));
      if (ftruncate(fd, static_cast<off_t>(size_)) != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("ftruncate failed: " + std::string(strerror(errno)));
      }
      map(fd);
      new (hdr()) Header();
      hdr()->magic = kMagic;
      hdr()->n_slots = n_slots;
      hdr()->slot_bytes = slot_bytes;
      hdr()->doorbell.store(0);
      hdr()->closed.store(0);
      for (uint32_t i = 0; i < n_slots; ++i) {
        Slot* s = new (slot(i)) Slot();
        s->req_seq.store(0);
        s->resp_seq.store(0);
        s->req_len.store(0);
        s->resp_len.store(0);
        s->pid.store(0);
        s->tag.store(0);
      }
    } else {
      int fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("shm_open(attach) failed for " + name + ": " + strerror(errno));
      struct stat st {};
      fstat(fd, &st);
      size_ = static_cast<size_t>(st.st_size);
      map(fd);
      if (hdr()->magic != kMagic) throw std::runtime_error("not an applestar shm channel: " + name);
    }
  }
  ~Segment() {
    if (base_) munmap(base_, size_);
    if (owner_) shm_unlink(name_.c_str());
  }
  Segment(const Segment&) = delete;
  Segment& operator=(const Segment&) = delete;

  static size_t layout_size(uint32_t n, uint64_t sb) {
    return slots_offset() + round_up(sizeof(Slot) * n, kPage) + 2 * sb * n;
  }
  static size_t slots_offset() { return round_up(sizeof(Header), kPage); }
  Header* hdr() const { return reinterpret_cast<Header*>(base_); }
  Slot* slot(uint32_t i) const {
    return reinterpret_cast<Slot*>(static_cast<char*>(base_) + slots_offset()) + i;
  }
  char* region(uint32_t i, bool response) const {
    const size_t data0 = slots_offset() + round_up(sizeof(Slot) * hdr()->n_slots, kPage);
    return static_cast<char*>(base_) + data0 + (2 * static_cast<size_t>(i) + (response ? 1 : 0)) * hdr()->slot_bytes;
  }
  uint32_t n_slots() const { return hdr()->n_slots; }
  uint64_t slot_bytes() const { return hdr()->slot_bytes; }
  void* base() const { return base_; }
  size_t size() const { return size_; }
  const std::string& name() const { return name_; }

 private:
  void map(int fd) {
    base_ = mmap(nullptr, size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (base_ == MAP_FAILED) {
      base_ = nullptr;
      throw std::runtime_error("mmap failed: " + std::string(strerror(errno)));
    }
  }
  std::string name_;
  bool owner_;
  void* base_ = nullptr;
  size_t size_ = 0;
};


enum class Wait { kOk = 0, kClosed = 1, kTimeout = 2 };

class ServerCore {
 public:
  ServerCore(const std::string& name, uint32_t n_slots, uint64_t slot_bytes)
      : seg_(name, n_slots, slot_bytes, true), served_(n_slots, 0) {}

  std::vector<uint32_t> pending() const {
    std::vector<uint32_t> ready;
    for (uint32_t i = 0; i < seg_.n_slots(); ++i)
      if (seg_.slot(i)->req_seq.load(std::memory_order_acquire) != served_[i]) ready.push_back(i);
    return ready;
  }

  // Slots with an unanswered request; blocks up to timeout_ms (-1 = forever) for the first one.
  std::vector<uint32_t> wait(int timeout_ms) const {
    const int64_t deadline = timeout_ms < 0 ? INT64_MAX : now_ms() + timeout_ms;
    while (true) {
      const uint32_t bell = seg_.hdr()->doorbell.load(std::memory_order_acquire);
      std::vector<uint32_t> ready = pending();
      if (!ready.empty() || seg_.hdr()->closed.load()) return ready;
      const int64_t left = deadline - now_ms();
      if (left <= 0) return ready;
      futex_wait(&seg_.hdr()->doorbell, bell, static_cast<int>(std::min<int64_t>(left, INT_MAX)));
    }
  }

  bool has_request(uint32_t i) const { return seg_.slot(i)->req_seq.load(std::memory_order_acquire) != served_[i]; }
  const char* request_data(uint32_t i) const { return seg_.region(i, false); }
  size_t request_len(uint32_t i) const { return seg_.slot(i)->req_len.load(std::memory_order_relaxed); }
  uint32_t tag(uint32_t i) const { return seg_.slot(i)->tag.load(std::memory_order_relaxed); }

  void respond(uint32_t i, const void* data, size_t n) {
    if (n > seg_.slot_bytes()) throw std::length_error("response larger than the slot");
    Slot* s = seg_.slot(i);
    const uint32_t seq = s->req_seq.load(std::memory_order_acquire);
    if (seq == served_[i]) throw std::runtime_error("respond without a pending request");
    std::memcpy(seg_.region(i, true), data, n);
    s->resp_len.store(n, std::memory_order_relaxed);
    s->resp_seq.store(seq, std::memory_order_release);
    served_[i] = seq;
    futex_wake(&s->resp_seq, INT_MAX);
  }

  std::vector<uint32_t> dead_slots() const {
    std::vector<uint32_t> out;
    for (uint32_t i = 0; i < seg_.n_slots(); ++i) {
      const int32_t pid = seg_.slot(i)->pid.load();
      if (pid > 0 && kill(pid, 0) != 0 && errno == ESRCH) out.push_back(i);
    }
    return out;
  }

  void close() {
    seg_.hdr()->closed.store(1);
    futex_wake(&seg_.hdr()->doorbell, INT_MAX);
    for (uint32_t i = 0; i < seg_.n_slots(); ++i) futex_wake(&seg_.slot(i)->resp_seq, INT_MAX);
  }

  const Segment& segment() const { return seg_; }

 private:
  Segment seg_;
  std::vector<uint32_t> served_;  // server-private: last answered request sequence per slot
};

class ClientCore {
 public:
  // owner_id: the pid recorded in the slot (threads of one process may pass distinct ids in tests)
  ClientCore(const std::string& name, uint32_t slot, uint32_t tag, int32_t owner_id = 0)
      : seg_(name, 0, 0, false), i_(slot), owner_(owner_id ? owner_id : static_cast<int32_t>(getpid())) {
    if (slot >= seg_.n_slots()) throw std::out_of_range("slot index");
    Slot* s = seg_.slot(i_);
    int32_t expect = 0;
    if (!s->pid.compare_exchange_strong(expect, owner_) && expect != owner_) {
      if (kill(expect, 0) == 0 || errno != ESRCH)
        throw std::runtime_error("slot " + std::to_string(slot) + " is owned by live pid " + std::to_string(expect));
      s->pid.store(owner_);  // previous owner died: take over
    }
    s->tag.store(tag);
    seq_ = s->req_seq.load();  // a response in flight for a dead predecessor is superseded by our request
  }
  ~ClientCore() {
    int32_t me = owner_;
    seg_.slot(i_)->pid.compare_exchange_strong(me, 0);
  }
  ClientCore(const ClientCore&) = delete;
  ClientCore& operator=(const ClientCore&) = delete;

  // Send one request and block for its response; on kOk the response is at response_data()/len.
  Wait request(const void* data, size_t n, int timeout_ms) {
    if (n > seg_.slot_bytes()) throw std::length_error("request larger than the slot");
    Slot* s = seg_.slot(i_);
    const uint32_t seq = ++seq_;  // a late response to an abandoned request is superseded by the next one
    std::memcpy(seg_.region(i_, false), data, n);
    s->req_len.store(n, std::memory_order_relaxed);
    s->req_seq.store(seq, std::memory_order_release);
    seg_.hdr()->doorbell.fetch_add(1, std::memory_order_acq_rel);
    futex_wake(&seg_.hdr()->doorbell, 1);
    const int64_t deadline = timeout_ms < 0 ? INT64_MAX : now_ms() + timeout_ms;
    while (true) {
      const uint32_t r = s->resp_seq.load(std::memory_order_acquire);
      if (r == seq) return Wait::kOk;
      if (seg_.hdr()->closed.load()) return Wait::kClosed;
      const int64_t left = deadline - now_ms();
      if (left <= 0) return Wait::kTimeout;
      futex_wait(&s->resp_seq, r, static_cast<int>(std::min<int64_t>(left, INT_MAX)));
    }
  }
  const char* response_data() const { return seg_.region(i_, true); }
  size_t response_len() const { return seg_.slot(i_)->resp_len.load(std::memory_order_relaxed); }
  uint32_t slot() const { return i_; }
  uint64_t slot_bytes() const { return seg_.slot_bytes(); }

 private:
  Segment seg_;
  uint32_t i_;
  int32_t owner_;
  uint32_t seq_ = 0;
};

}  // namespace as_host
