// fdcn_session_book.h -- host-only bookkeeping of a device session
// (fdcn_session.hip), kept free of HIP calls so `make asan` can instrument
// it on the CPU (tools/sanitize/session_book_driver.cpp):
//   Layout        offsets of 256-byte-aligned sub-buffers of one staging block
//   PinnedArenaT  the bump allocator over pinned chunks that stages every
//                 call's host arrays (the allocator is a template parameter:
//                 hipHostMalloc in the library, malloc in the driver)
//   SlotTable     slot number -> device vector, its length and the event of
//                 the launch that produced it; argument checks; the distinct
//                 producer events a consumer must wait for
// Nothing here is thread-safe: a session belongs to one thread (fdcn.h).
#ifndef FDCN_SESSION_BOOK_H
#define FDCN_SESSION_BOOK_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

namespace fdcn_book {

inline size_t al256(size_t n) { return (n + 255) / 256 * 256; }

struct Layout {
  size_t size = 0;
  size_t add(size_t bytes) {
    const size_t o = size;
    size += al256(bytes > 0 ? bytes : 1);
    return o;
  }
};

// Bump allocation over chunks of at least 8 MB.  Within a session every
// region handed out stays untouched by later calls of that session (async
// copies may still read it); reset() recycles everything and is called only
// after the session's streams have drained.  trim(keep) releases the chunks
// beyond the first `keep` bytes (after reset: nothing in use).
template <class Alloc>
struct PinnedArenaT {
  struct Chunk {
    char* p;
    size_t cap;
  };
  std::vector<Chunk> chunks;
  size_t cur = 0, used = 0;

  char* get(size_t bytes) {
    bytes = al256(bytes > 0 ? bytes : 1);
    while (cur < chunks.size() && used + bytes > chunks[cur].cap) {
      ++cur;
      used = 0;
    }
    if (cur == chunks.size()) {
      const size_t sz = std::max(bytes, (size_t)8 << 20);
      char* p = static_cast<char*>(Alloc::alloc(sz));
      if (!p) return nullptr;
      chunks.push_back({p, sz});
      used = 0;
    }
    char* r = chunks[cur].p + used;
    used += bytes;
    return r;
  }
  // [p, p + n) lies inside one chunk this arena holds (a region it handed
  // out: pinned memory an async copy may read directly)
  bool owns(const void* p, size_t n) const {
    const char* c = static_cast<const char*>(p);
    for (const Chunk& k : chunks)
      if (c >= k.p && n <= k.cap && c - k.p <= (ptrdiff_t)(k.cap - n)) return true;
    return false;
  }
  void reset() { cur = used = 0; }
  void trim(size_t keep) {
    size_t held = 0, k = 0;
    while (k < chunks.size() && held + chunks[k].cap <= keep) held += chunks[k++].cap;
    for (size_t i = k; i < chunks.size(); ++i) Alloc::release(chunks[i].p);
    chunks.resize(k);
    if (cur > chunks.size()) cur = chunks.size();
  }
  size_t bytes_held() const {
    size_t s = 0;
    for (const Chunk& c : chunks) s += c.cap;
    return s;
  }
};

struct SlotTable {
  std::vector<double*> ptr;
  std::vector<int32_t> n;
  std::vector<int32_t> ev;

  int32_t size() const { return (int32_t)ptr.size(); }

  // 0, or writes the reason to err and returns -1: a slot number outside
  // the table, or one holding another length (n_nodes < 0: any length)
  int check(int32_t count, const int32_t* slots, int32_t n_nodes, char* err,
            size_t errlen) const {
    for (int32_t i = 0; i < count; ++i) {
      const int32_t k = slots[i];
      if (k < 0 || k >= size()) {
        snprintf(err, errlen, "slot %d does not exist (session has %d)", k, size());
        return -1;
      }
      if (n_nodes >= 0 && n[(size_t)k] != n_nodes) {
        snprintf(err, errlen, "slot %d holds %d nodes, expected %d", k, n[(size_t)k], n_nodes);
        return -1;
      }
    }
    return 0;
  }

  // B consecutive vectors of n_nodes doubles from `base`, produced by event
  // `event`: their slot numbers into out[B]
  void add(double* base, int32_t B, int32_t n_nodes, int32_t event, int32_t* out) {
    for (int32_t b = 0; b < B; ++b) {
      out[b] = size();
      ptr.push_back(base + (size_t)b * n_nodes);
      n.push_back(n_nodes);
      ev.push_back(event);
    }
  }

  // the distinct events that produced `slots` (checked), ascending
  std::vector<int32_t> producers(int32_t count, const int32_t* slots) const {
    std::vector<int32_t> evs;
    evs.reserve((size_t)count);
    for (int32_t i = 0; i < count; ++i) evs.push_back(ev[(size_t)slots[i]]);
    std::sort(evs.begin(), evs.end());
    evs.erase(std::unique(evs.begin(), evs.end()), evs.end());
    return evs;
  }
};

}  // namespace fdcn_book

#endif  // FDCN_SESSION_BOOK_H
