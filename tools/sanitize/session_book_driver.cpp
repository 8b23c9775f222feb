// session_book_driver.cpp -- CPU driver of the device sessions' host-only
// bookkeeping (finite_difference_amd/csrc/fdcn_session_book.h) for the
// sanitizer build (`make asan`: AddressSanitizer + UndefinedBehaviorSanitizer,
// first report aborts).  The library
// instantiates the arena over hipHostMalloc; here over malloc, so every
// chunk is visible to ASan.  The driver replays the call patterns of
// fdcn_session.hip -- staging blocks of every size class through the arena
// (a whole-file plan's hundreds of MB, a trade's few KB), slot creation,
// checks and producer-event queries, the destroy path's reset + trim back
// to the idle cap, and a reused context -- writing every byte it is handed
// and checking every answer.  Exit 0 = clean.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../finite_difference_amd/csrc/fdcn_session_book.h"

namespace {

int g_allocs = 0, g_frees = 0;

struct MallocAlloc {
  static void* alloc(size_t n) {
    ++g_allocs;
    return malloc(n);
  }
  static void release(void* p) {
    ++g_frees;
    free(p);
  }
};

#define CHECK(c)                                                          \
  do {                                                                    \
    if (!(c)) {                                                           \
      fprintf(stderr, "session_book_driver: %s:%d: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

void test_layout() {
  fdcn_book::Layout L;
  CHECK(L.add(0) == 0 && L.size == 256);
  CHECK(L.add(1) == 256 && L.size == 512);
  CHECK(L.add(257) == 512 && L.size == 1024);
}

// one session's worth of staging: regions never overlap while "in use"
void session_round(fdcn_book::PinnedArenaT<MallocAlloc>& arena, unsigned seed, size_t big) {
  std::vector<std::pair<char*, size_t>> live;
  for (int call = 0; call < 40; ++call) {
    seed = seed * 1103515245u + 12345u;
    size_t n = (seed >> 8) % 70000;
    if (call % 13 == 5) n = big;  // a whole-file plan's staging
    char* p = arena.get(n);
    CHECK(p != nullptr);
    CHECK(((uintptr_t)p & 255) == 0);
    memset(p, call & 0xff, n ? n : 1);  // every byte handed out is writable
    for (auto& r : live)                // and disjoint from the live regions
      CHECK(p + (n ? n : 1) <= r.first || r.first + (r.second ? r.second : 1) <= p);
    live.push_back({p, n});
    CHECK(arena.owns(p, n ? n : 1));  // a handed-out region is pinned memory
  }
  for (size_t i = 0; i < live.size(); ++i)  // nothing was overwritten since
    if (live[i].second) CHECK((unsigned char)live[i].first[live[i].second - 1] == (i & 0xff));
}

void test_owns() {
  fdcn_book::PinnedArenaT<MallocAlloc> arena;
  char* p = arena.get(1000);
  const size_t cap = arena.chunks[0].cap;
  CHECK(arena.owns(p, 1000) && arena.owns(p + 17, 983) && arena.owns(p, cap));
  CHECK(!arena.owns(p, cap + 1) && !arena.owns(p + cap, 1) && !arena.owns(p - 1, 8));
  std::vector<double> heap(64);  // caller memory that is not the arena's
  CHECK(!arena.owns(heap.data(), sizeof(double) * heap.size()));
  arena.reset();
  arena.trim(0);
}

void test_arena() {
  fdcn_book::PinnedArenaT<MallocAlloc> arena;
  const size_t keep = (size_t)24 << 20;
  session_round(arena, 1, (size_t)40 << 20);
  CHECK(arena.bytes_held() >= ((size_t)40 << 20));
  arena.reset();  // fdcn_session_destroy after the streams drained
  arena.trim(keep);
  CHECK(arena.bytes_held() <= keep);
  session_round(arena, 2, (size_t)3 << 20);  // the context reused by the next session
  arena.reset();
  arena.trim(0);
  CHECK(arena.chunks.empty() && arena.bytes_held() == 0);
  CHECK(g_allocs == g_frees);
}

void test_slots() {
  fdcn_book::SlotTable t;
  std::vector<double> a(3 * 17), b(2 * 9);
  int32_t out[3];
  t.add(a.data(), 3, 17, 0, out);
  CHECK(out[0] == 0 && out[2] == 2 && t.size() == 3 && t.ptr[2] == a.data() + 34);
  t.add(b.data(), 2, 9, 1, out);
  CHECK(out[0] == 3 && out[1] == 4 && t.n[4] == 9 && t.ev[4] == 1);
  char err[160];
  const int32_t ok[3] = {0, 2, 1};
  CHECK(t.check(3, ok, 17, err, sizeof(err)) == 0);
  const int32_t missing[2] = {1, 5};
  CHECK(t.check(2, missing, 17, err, sizeof(err)) == -1 && strstr(err, "does not exist"));
  const int32_t neg[1] = {-1};
  CHECK(t.check(1, neg, -1, err, sizeof(err)) == -1);
  const int32_t wrong[2] = {0, 3};
  CHECK(t.check(2, wrong, 17, err, sizeof(err)) == -1 && strstr(err, "holds 9 nodes"));
  CHECK(t.check(2, wrong, -1, err, sizeof(err)) == 0);
  const int32_t mixed[5] = {4, 0, 3, 1, 0};
  const std::vector<int32_t> ev = t.producers(5, mixed);
  CHECK(ev.size() == 2 && ev[0] == 0 && ev[1] == 1);
  CHECK(t.producers(0, mixed).empty());
  for (int32_t k = 0; k < t.size(); ++k) t.ptr[(size_t)k][0] = (double)k;  // slots address live memory
  CHECK(a[17] == 1.0 && b[9] == 4.0);
}

}  // namespace

int main() {
  test_layout();
  test_owns();
  test_arena();
  test_slots();
  printf("session_book_driver: ok\n");
  return 0;
}
