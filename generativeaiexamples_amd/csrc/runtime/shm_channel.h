// Single-writer / multi-reader broadcast ring in POSIX shared memory.
//
// A tensor-parallel engine has ONE scheduler (rank 0). Every step it serialises the step plan (token
// ids, positions, KV slots, block tables, sampling parameters) and broadcasts it to the follower
// ranks, which execute exactly the same forward / collectives. All ranks of a TP group live on one
// MI355X node, so the plan travels through host shared memory instead of a collective: a publish is a
// memcpy plus one release store, a follower picks it up within microseconds of spinning, and nothing
// is queued on the GPU streams (the RCCL streams stay free for the forward's all-reduces).
//
// Layout: [Header][slot 0]...[slot n-1]; each slot = [SlotHdr][payload of slot_bytes]. Sequence numbers
// start at 1. The writer may reuse slot (s mod n) for message s only after every reader has consumed
// message s - n (reader cursors live in the header on separate cache lines). Readers spin, then back off
// to short sleeps; they give up with an error when the writer process has died (kill(pid, 0)) or an
// optional timeout expires, so a crashed rank 0 never leaves followers hanging forever.
#pragma once

#include <atomic>
#include <cstdint>
#include <string>
#include <vector>

namespace gai {

class ShmChannel {
 public:
  static constexpr int kMaxReaders = 64;

  // writer: creates (and unlinks on destruction) the segment
  static ShmChannel* create(const std::string& name, int num_readers, uint64_t slot_bytes, int num_slots);
  // reader `reader` (0 .. num_readers-1): opens an existing segment (waits up to timeout_s for it)
  static ShmChannel* open(const std::string& name, int reader, double timeout_s);
  ~ShmChannel();

  // writer: publish one message (blocks while the oldest slot is still unread; -> false on timeout)
  bool send(const char* data, uint64_t len, double timeout_s);
  // reader: next message into `out` (-> 0 ok, 1 timeout, 2 writer gone)
  int recv(std::vector<char>& out, double timeout_s);

  uint64_t slot_bytes() const;
  int num_readers() const;
  uint64_t sent() const;

  struct Header;
  struct SlotHdr;

 private:
  ShmChannel() = default;
  char* slot(uint64_t seq) const;
  std::string name_;
  char* base_ = nullptr;
  uint64_t size_ = 0;
  int reader_ = -1;  // -1 = writer
  uint64_t next_ = 1;
  bool owner_ = false;
};

}  // namespace gai
