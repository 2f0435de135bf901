// POSIX shared-memory broadcast ring: see shm_channel.h.
#include "shm_channel.h"

#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>
#include <thread>

namespace gai {

namespace {
constexpr uint64_t kMagic = 0x47414953484d4331ull;  // "GAISHMC1"
constexpr uint64_t kLine = 128;

double now_s() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

// spin -> yield -> sleep backoff, by iteration count
void backoff(uint64_t it) {
  if (it < 2000) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  } else if (it < 4000) {
    sched_yield();
  } else {
    std::this_thread::sleep_for(std::chrono::microseconds(it < 20000 ? 20 : 200));
  }
}
}  // namespace

struct alignas(kLine) ShmChannel::Header {
  uint64_t magic;
  uint64_t slot_bytes;
  int32_t num_slots;
  int32_t num_readers;
  int32_t writer_pid;
  int32_t pad0;
  alignas(kLine) std::atomic<uint64_t> sent;  // messages published
  struct alignas(kLine) Cursor {
    std::atomic<uint64_t> done;  // last message this reader consumed
  } cursor[kMaxReaders];
};

struct alignas(kLine) ShmChannel::SlotHdr {
  std::atomic<uint64_t> seq;  // message number held by this slot (0 = never written)
  uint64_t len;
};

static uint64_t slot_stride(uint64_t slot_bytes) {
  return (sizeof(ShmChannel::SlotHdr) + slot_bytes + kLine - 1) / kLine * kLine;
}

char* ShmChannel::slot(uint64_t seq) const {
  const Header* h = reinterpret_cast<const Header*>(base_);
  return base_ + sizeof(Header) + ((seq - 1) % (uint64_t)h->num_slots) * slot_stride(h->slot_bytes);
}

ShmChannel* ShmChannel::create(const std::string& name, int num_readers, uint64_t slot_bytes, int num_slots) {
  if (num_readers < 0 || num_readers > kMaxReaders || num_slots < 1 || slot_bytes == 0)
    throw std::invalid_argument("ShmChannel: bad geometry");
  const uint64_t size = sizeof(Header) + (uint64_t)num_slots * slot_stride(slot_bytes);
  shm_unlink(name.c_str());  // a stale segment of a crashed run
  int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("ShmChannel: shm_open(create) failed: " + std::string(strerror(errno)));
  if (ftruncate(fd, (off_t)size) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error("ShmChannel: ftruncate failed");
  }
  void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    throw std::runtime_error("ShmChannel: mmap failed");
  }
  std::memset(p, 0, sizeof(Header));
  auto* ch = new ShmChannel();
  ch->name_ = name;
  ch->base_ = static_cast<char*>(p);
  ch->size_ = size;
  ch->owner_ = true;
  Header* h = reinterpret_cast<Header*>(p);
  h->slot_bytes = slot_bytes;
  h->num_slots = num_slots;
  h->num_readers = num_readers;
  h->writer_pid = (int32_t)getpid();
  for (int s = 0; s < num_slots; ++s) {
    auto* sh = reinterpret_cast<SlotHdr*>(ch->base_ + sizeof(Header) + (uint64_t)s * slot_stride(slot_bytes));
    sh->seq.store(0, std::memory_order_relaxed);
    sh->len = 0;
  }
  h->sent.store(0, std::memory_order_relaxed);
  for (int r = 0; r < kMaxReaders; ++r) h->cursor[r].done.store(0, std::memory_order_relaxed);
  std::atomic_thread_fence(std::memory_order_release);
  reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->store(kMagic, std::memory_order_release);
  return ch;
}

ShmChannel* ShmChannel::open(const std::string& name, int reader, double timeout_s) {
  const double t0 = now_s();
  int fd = -1;
  for (uint64_t it = 0;; ++it) {
    fd = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd >= 0) {
      struct stat st;
      if (fstat(fd, &st) == 0 && (uint64_t)st.st_size >= sizeof(Header)) break;
      close(fd);
      fd = -1;
    }
    if (timeout_s >= 0 && now_s() - t0 > timeout_s) throw std::runtime_error("ShmChannel: open timed out: " + name);
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  struct stat st;
  fstat(fd, &st);
  void* p = mmap(nullptr, (size_t)st.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error("ShmChannel: mmap failed");
  Header* h = reinterpret_cast<Header*>(p);
  for (uint64_t it = 0; reinterpret_cast<std::atomic<uint64_t>*>(&h->magic)->load(std::memory_order_acquire) != kMagic;
       ++it) {
    if (timeout_s >= 0 && now_s() - t0 > timeout_s) {
      munmap(p, (size_t)st.st_size);
      throw std::runtime_error("ShmChannel: segment never initialised: " + name);
    }
    backoff(it);
  }
  if (reader < 0 || reader >= h->num_readers) {
    munmap(p, (size_t)st.st_size);
    throw std::invalid_argument("ShmChannel: reader index out of range");
  }
  auto* ch = new ShmChannel();
  ch->name_ = name;
  ch->base_ = static_cast<char*>(p);
  ch->size_ = (uint64_t)st.st_size;
  ch->reader_ = reader;
  ch->next_ = h->cursor[reader].done.load(std::memory_order_acquire) + 1;
  return ch;
}

ShmChannel::~ShmChannel() {
  if (base_) munmap(base_, size_);
  if (owner_) shm_unlink(name_.c_str());
}

uint64_t ShmChannel::slot_bytes() const { return reinterpret_cast<const Header*>(base_)->slot_bytes; }
int ShmChannel::num_readers() const { return reinterpret_cast<const Header*>(base_)->num_readers; }
uint64_t ShmChannel::sent() const { return reinterpret_cast<const Header*>(base_)->sent.load(std::memory_order_acquire); }

bool ShmChannel::send(const char* data, uint64_t len, double timeout_s) {
  if (reader_ != -1) throw std::logic_error("ShmChannel: send() on a reader");
  Header* h = reinterpret_cast<Header*>(base_);
  if (len > h->slot_bytes) throw std::length_error("ShmChannel: message larger than the slot");
  const uint64_t seq = next_;
  // slot reuse: every reader must have consumed message seq - num_slots
  if (seq > (uint64_t)h->num_slots) {
    const uint64_t need = seq - (uint64_t)h->num_slots;
    const double t0 = now_s();
    for (int r = 0; r < h->num_readers; ++r) {
      for (uint64_t it = 0; h->cursor[r].done.load(std::memory_order_acquire) < need; ++it) {
        if (timeout_s >= 0 && (it & 255) == 0 && now_s() - t0 > timeout_s) return false;
        backoff(it);
      }
    }
  }
  SlotHdr* sh = reinterpret_cast<SlotHdr*>(slot(seq));
  std::memcpy(reinterpret_cast<char*>(sh) + sizeof(SlotHdr), data, len);
  sh->len = len;
  sh->seq.store(seq, std::memory_order_release);
  h->sent.store(seq, std::memory_order_release);
  ++next_;
  return true;
}

int ShmChannel::recv(std::vector<char>& out, double timeout_s) {
  if (reader_ < 0) throw std::logic_error("ShmChannel: recv() on the writer");
  Header* h = reinterpret_cast<Header*>(base_);
  const uint64_t seq = next_;
  SlotHdr* sh = reinterpret_cast<SlotHdr*>(slot(seq));
  const double t0 = now_s();
  for (uint64_t it = 0; sh->seq.load(std::memory_order_acquire) != seq; ++it) {
    if ((it & 1023) == 1023) {
      if (kill(h->writer_pid, 0) != 0 && errno == ESRCH) return 2;
      if (timeout_s >= 0 && now_s() - t0 > timeout_s) return 1;
    }
    backoff(it);
  }
  out.assign(reinterpret_cast<char*>(sh) + sizeof(SlotHdr), reinterpret_cast<char*>(sh) + sizeof(SlotHdr) + sh->len);
  h->cursor[reader_].done.store(seq, std::memory_order_release);
  ++next_;
  return 0;
}

}  // namespace gai
