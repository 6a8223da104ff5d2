// ring_protocol_test.cpp — CPU model check of the resident encoder's ring protocol (tests only).
//
// Uses the product's own definitions (fec_kernels.hpp: ServerSlot / ServerControl / ServerCoord
// layout, server_tag, server_scrub_after, the inline chunk constants) and checks the properties
// the server's and the host's acceptance rules rest on (DESIGN_HISTORY.md §8c round 5):
//  1. tags: 1 .. epoch, never 0 (the zeroed state); a slot's tags over `epoch` consecutive laps are
//     all different; the scrub falls on the last lap of every epoch;
//  2. no stale acceptance: a slot modelled over many laps at 8-B granularity -- the host's halves
//     land in any order, some only after the server looked (torn write-combined stores), words of
//     the previous laps stay where a later call did not overwrite them, the server zeroes the slot
//     after the last lap of an epoch -- is never accepted by the server's rule (every half it
//     reads carries tag(seq)) unless every half it reads is this lap's;
//  3. serving classes: with per-class seq counters (class c takes c, c + K, c + 2K, ...; the host's
//     choice by calls in flight) every class's seqs map to slots of that class only
//     (seq % kServerSlots), and a slot's previous occupant is always seq - kServerSlots;
//  4. layout: the structures' sizes the host, the device and the inline data area assume;
//  5. leaving as a whole: the workgroups of one instance share idle flags, a leave
//     word and an exit count (ServerCoord, server_all_idle / server_exits_next / server_exits_last)
//     -- modelled over thousands of instances with random interleavings, workgroups dispatched
//     late (after another one set the leave word), the host's stop word and the previous
//     instance's words left in place: every workgroup leaves within its next coordination read
//     once the leave word is set, none leaves on an earlier instance's words, and exactly one
//     workgroup per instance -- the last to count out -- stores exited = gen.  Controls with the
//     generation checks removed must fail.
// Prints "OK <checks>" or the first violation.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <vector>

#include "fec_kernels.hpp"

using namespace qfec;

static long g_checks = 0;
#define CHECK(cond, ...)                     \
  do {                                       \
    ++g_checks;                              \
    if (!(cond)) {                           \
      std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);              \
      std::printf("\n");                     \
      std::exit(1);                          \
    }                                        \
  } while (0)

static void tags() {
  for (uint32_t epoch : {1u, 2u, 4u, 128u, kServerEpoch}) {
    for (uint64_t base_lap : {0ull, 7ull, 32767ull, 1ull << 20}) {
      std::set<uint32_t> seen;
      for (uint64_t lap = base_lap; lap < base_lap + epoch; ++lap) {
        const uint64_t seq = lap * kServerSlots + 5;
        const uint32_t t = server_tag(seq, epoch);
        CHECK(t >= 1 && t <= epoch, "tag %u outside 1..%u", t, epoch);
        CHECK(seen.insert(t).second, "tag %u repeats within %u laps", t, epoch);
        CHECK(server_scrub_after(seq, epoch) == ((lap % epoch) == epoch - 1), "scrub at lap %llu epoch %u",
              (unsigned long long)lap, epoch);
        CHECK(t < (1u << 16), "tag %u does not fit 16 bits", t);
      }
    }
  }
}

// One slot of inline halves (the model's unit: 8-B words), written lap after lap.  scrub: the
// server zeroes the slot after the last lap of each epoch (the product); without it (the control)
// a word left from an earlier epoch carries the current tag again.  Returns the stale acceptances.
static long stale_acceptances(bool scrub) {
  long stale = 0;
  std::mt19937_64 rng(0x5EEDu);
  for (uint32_t epoch : {2u, 4u, 32u}) {
    constexpr uint32_t kWords = 24;           // halves of the slot's data area the calls use
    std::vector<uint32_t> word_tag(kWords, 0);  // tag in each word's top 16 bits (0 = zeroed)
    std::vector<uint64_t> word_lap(kWords, ~0ull);
    for (uint64_t lap = 0; lap < 40ull * epoch; ++lap) {
      const uint64_t seq = lap * kServerSlots + 3;
      const uint32_t tag = server_tag(seq, epoch);
      // this call writes the first n words (shorter calls leave older words in place)
      const uint32_t n = 1 + static_cast<uint32_t>(rng() % kWords);
      std::vector<uint32_t> order(n);
      for (uint32_t i = 0; i < n; ++i) order[i] = i;
      std::shuffle(order.begin(), order.end(), rng);
      // the server may look after any number of the call's words have landed
      const uint32_t landed_at_look = static_cast<uint32_t>(rng() % (n + 1));
      for (uint32_t k = 0; k <= n; ++k) {
        if (k == landed_at_look) {
          // the server's rule: every word it reads (the call's n) carries this lap's tag
          bool accept = true;
          for (uint32_t w = 0; w < n; ++w) accept = accept && word_tag[w] == tag;
          bool all_current = true;
          for (uint32_t w = 0; w < n; ++w) all_current = all_current && word_lap[w] == lap;
          if (accept && !all_current) {
            ++stale;
          } else if (scrub) {
            CHECK(accept == (k == n), "epoch %u lap %llu: acceptance %d with %u of %u words landed", epoch,
                  (unsigned long long)lap, int(accept), k, n);
          }
        }
        if (k < n) {
          word_tag[order[k]] = tag;
          word_lap[order[k]] = lap;
        }
      }
      // served: at the last lap of an epoch the server zeroes the slot before its done word
      if (scrub && server_scrub_after(seq, epoch)) {
        std::fill(word_tag.begin(), word_tag.end(), 0u);
        std::fill(word_lap.begin(), word_lap.end(), ~0ull);
      }
    }
  }
  return stale;
}

static void classes() {
  for (uint32_t K : {1u, 2u, 4u, 8u}) {
    CHECK(kServerSlots % K == 0, "%u classes do not divide the slots", K);
    std::vector<uint64_t> next(K);
    for (uint32_t c = 0; c < K; ++c) next[c] = c;
    std::vector<uint64_t> last_seq(kServerSlots, ~0ull);
    std::mt19937 rng(K);
    for (int call = 0; call < 200000; ++call) {
      // the host's choice: round robin over the lowest min(K, in flight) classes
      const uint32_t in_flight = 1 + rng() % 16;
      const uint32_t span = in_flight < K ? in_flight : K;
      const uint32_t c = span > 1 ? static_cast<uint32_t>(call) % span : 0u;
      const uint64_t seq = next[c];
      next[c] += K;
      const uint32_t si = static_cast<uint32_t>(seq % kServerSlots);
      CHECK(si % K == c, "class %u seq %llu in slot %u of class %u", c, (unsigned long long)seq, si, si % K);
      CHECK(seq % K == c, "class %u took seq %llu", c, (unsigned long long)seq);
      if (seq >= kServerSlots) {
        CHECK(last_seq[si] == seq - kServerSlots, "slot %u: previous occupant %llu, not %llu", si,
              (unsigned long long)last_seq[si], (unsigned long long)(seq - kServerSlots));
      } else {
        CHECK(last_seq[si] == ~0ull, "slot %u reused in the first lap", si);
      }
      last_seq[si] = seq;
    }
  }
}

static void layout() {
  CHECK(sizeof(ServerSlot) % 64 == 0 && sizeof(ServerSlot) >= 16 * 8, "ServerSlot %zu B", sizeof(ServerSlot));
  CHECK(sizeof(ServerControl) % 64 == 0, "ServerControl %zu B", sizeof(ServerControl));
  CHECK(sizeof(ServerCoord) % 64 == 0 && sizeof(ServerCoord) >= 16 + 8 * kServerMaxClasses, "ServerCoord %zu B",
        sizeof(ServerCoord));
  CHECK((kServerMaxClasses & (kServerMaxClasses - 1)) == 0 && kServerSlots % kServerMaxClasses == 0, "classes");
  CHECK(kInlinePayload == 12 && kInlineSlotBytes ==
            kInlineMaxGroups * kServerPackets * ((kInlineMaxP + kInlinePayload - 1) / kInlinePayload) * 16,
        "inline area %u B", kInlineSlotBytes);
  CHECK(kServerAddrMask == (1ull << 48) - 1 && (kServerEpoch & (kServerEpoch - 1)) == 0 && kServerEpoch <= 65535,
        "tag field");
  CHECK(kServerPoll * 16 / 2 + 2 + kServerMaxClasses / 2 <= 1024, "the poll's lanes fit the workgroup");
}

// 5. The coordination words, modelled.  One instance = K workgroups; a step runs one poll of one
// workgroup (its reads and stores of the shared words are the kernel's, each atomic) or one
// step of its exit count (the load, then CAS attempts).  Returns the violations found; with
// `control` != 0 the model runs a broken rule (1: the leave word read without its generation,
// 2: the exit count without the generation reset) and must find violations.
struct CoordModel {
  uint64_t leave = 0, exits = 0, idle[kServerMaxClasses] = {}, exited = 0;
};

static long coordination(int control, long* instances_out) {
  constexpr uint32_t kEvery = 8;    // the kernel reads the shared words every 8th poll (kCoordEvery + 1)
  constexpr uint32_t kMaxPolls = 4000;
  long violations = 0, instances = 0;
  std::mt19937_64 rng(0xC0DEu + control);
  for (uint32_t K : {2u, 4u, 8u}) {
    CoordModel m;  // a Resident's coordination words start zeroed (fec_coalesce.cpp hipMemsetAsync)
    for (uint64_t gen = 1; gen <= 1500; ++gen, ++instances) {
      // the host relaunches only once the previous instance's exited word is its generation
      if (m.exited != gen - 1) {
        ++violations;
        m.exited = gen - 1;
      }
      struct Wg {
        bool started = false, leaving = false, counted = false;
        uint32_t it = 0, t_last = 0, polls_after_leave = 0;
        bool told = false, was_idle = false;
        uint64_t idle_seen[kServerMaxClasses] = {};
        uint64_t v = 0;
        bool have_v = false;
      };
      std::vector<Wg> wg(K);
      // work per class: busy for a random number of polls (some classes none at all)
      std::vector<uint32_t> busy_until(K);
      for (auto& b : busy_until) b = static_cast<uint32_t>(rng() % 3 == 0 ? 0 : rng() % 200);
      const uint32_t idle_polls = 5 + static_cast<uint32_t>(rng() % 40);
      const uint32_t life_polls = rng() % 4 == 0 ? 30 + static_cast<uint32_t>(rng() % 200) : kMaxPolls;
      const bool host_stop = rng() % 8 == 0;
      const uint64_t stop_at_step = rng() % 3000;
      bool any_legit = false;   // a workgroup of this instance had a reason of its own to leave
      uint32_t exited_stores = 0, counted = 0;
      int last_counter = -1;
      uint64_t step = 0;
      for (; counted < K && step < 2000000; ++step) {
        const uint32_t c = static_cast<uint32_t>(rng() % K);
        Wg& w = wg[c];
        if (w.counted) continue;
        if (!w.started) {  // dispatched late: often long after the others
          if (rng() % 64 != 0) continue;
          w.started = true;
        }
        if (!w.leaving) {
          if (w.it % kEvery == 0) {
            w.told = control == 1 ? m.leave != 0 : m.leave == gen;
            for (uint32_t q = 0; q < K; ++q) w.idle_seen[q] = m.idle[q];
          }
          if (m.leave == gen) ++w.polls_after_leave;
          const bool work = w.it < busy_until[c];
          if (work) w.t_last = w.it;
          const bool idle = !work && w.it - w.t_last > idle_polls;
          const bool stop = host_stop && step >= stop_at_step;
          const bool own = stop || w.it > life_polls || w.it + 1 == kMaxPolls;
          const bool all_idle = server_all_idle(idle, w.idle_seen, K, c, gen);
          if (idle != w.was_idle) {
            m.idle[c] = idle ? gen : 0;
            w.was_idle = idle;
          }
          if (own || all_idle) any_legit = true;
          if ((own || all_idle) && !w.told) m.leave = gen;
          if (w.told && !any_legit) ++violations;  // left on an earlier instance's word
          w.leaving = own || all_idle || w.told;
          ++w.it;
          continue;
        }
        // counting out: the load, then CAS attempts (another workgroup may get in between)
        if (!w.have_v) {
          w.v = m.exits;
          w.have_v = true;
          continue;
        }
        const uint64_t nv = control == 2 ? w.v + 1 : server_exits_next(w.v, gen);
        if (m.exits != w.v) {
          w.v = m.exits;
          continue;
        }
        m.exits = nv;
        w.counted = true;
        ++counted;
        if (server_exits_last(nv, K)) {
          m.exited = gen;
          ++exited_stores;
          last_counter = static_cast<int>(c);
        }
      }
      if (counted != K) ++violations;           // a workgroup never left
      if (exited_stores != 1) ++violations;      // nobody, or more than one, stored exited
      if (last_counter >= 0) {
        for (uint32_t q = 0; q < K; ++q)
          if (static_cast<int>(q) != last_counter && !wg[q].counted) ++violations;
      }
      // once the leave word is this instance's, each workgroup leaves within one coordination read
      for (uint32_t q = 0; q < K; ++q)
        if (wg[q].polls_after_leave > kEvery + 1) ++violations;
      if (m.exited != gen) m.exited = gen;  // keep the next instance's precondition for the controls
    }
  }
  *instances_out = instances;
  return violations;
}

int main() {
  tags();
  const long with_scrub = stale_acceptances(true), without = stale_acceptances(false);
  CHECK(with_scrub == 0, "%ld stale acceptances with the epoch scrub", with_scrub);
  CHECK(without > 0, "the control (no scrub) found no stale acceptance: the model has no teeth");
  classes();
  layout();
  long instances = 0;
  const long bad = coordination(0, &instances);
  CHECK(bad == 0, "%ld coordination violations over %ld instances", bad, instances);
  CHECK(coordination(1, &instances) > 0, "control 1 (leave word without generation) found nothing");
  CHECK(coordination(2, &instances) > 0, "control 2 (exit count without generation reset) found nothing");
  std::printf("OK %ld\n", g_checks);
  return 0;
}
