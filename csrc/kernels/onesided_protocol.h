// One-sided THRESHOLD rounds over mapped peer windows: the protocol.
//
// This header is the single definition of the lane's rules.  The gfx950
// kernels (onesided.hip) and the CPU backend (transport/onesided.cpp, windows
// in POSIX shared memory, one process per rank) both run these functions, so
// the CPU tests exercise exactly the decisions the GPU makes.
//
// What it reproduces (reference AllreduceWorker.scala):
//  * fire-and-forget sends: every ScatterBlock / ReduceBlock is a `!`
//    (W:227-232, W:259-264) -- here a store into the receiver's window that
//    never waits for the receiver;
//  * reduce at thReduce: a chunk is summed as soon as floor(thReduce * N)
//    copies landed, over exactly the landed set, count = popcount
//    (SB:9-13, SB:20-32, W:177-181);
//  * complete at thComplete: a round completes once floor(thComplete * total)
//    reduced chunks landed; missing chunks are 0 with count 0 (RB:13-17,
//    RB:26-53, RB:60-66);
//  * outdated messages are dropped (W:155-156, W:172-173) -- here the SENDER
//    skips a push the receiver can no longer use (it already reduced that
//    chunk / completed that round), so the bytes never cross the link;
//  * bounded staleness: a round older than (latest round any peer pushed to
//    me) - maxLag is force-reduced / force-completed with what landed
//    (catch-up, W:100-106), and a call starts no earlier than that round
//    (implicit start of future rounds, W:164-167 / W:182-185);
//  * liveness: a wait never depends on a copy that cannot come any more -- a
//    source that announced a later round, or retired, is past round r
//    (source_past), so "landed + still possible < needed" ends the wait.
//
// Memory of a rank (its "window", mapped by every peer):
//   scatter rows  SD[row][src][slot]   src's contribution to my block
//   gather rows   GD[row][blk][slot]   block blk's reduced chunks (pushed by blk)
//   flag words    (below)
// with row = round % D.  D is the transport's ring depth, independent of
// maxLag: any D >= 2 is correct, larger D only loses fewer late messages.
//
// Tags.  Every (row, src, chunk, part) of SD and (row, blk, chunk, part) of
// GD has ONE writer (src, resp. blk), which writes rounds in increasing
// order.  Its tag word says which round the bytes belong to:
//   2(r+1)     writing round r (marker stored BEFORE the data)
//   2(r+1)+1   round r complete (stored after the data, behind a release)
// A reader trusts bytes only under a "done r" tag.  A tag of a later round
// means the writer moved past r: that copy of round r is lost for good.
//
// Overwrite hand-shake.  A writer of round x may find the reader still
// reading the same row for an older round y < x (the reader is >= D rounds
// behind).  Both sides announce, then look (store -> full fence -> load):
//   reader: sread[row][chunk] = y+1 (resp. gread[row]); then reads tags;
//   writer: tag = "writing x"; then reads sread / gread; if it shows an
//           older round in progress, the write is dropped (tag stays
//           "writing x": never mistaken for data).
// Either the writer sees the reader's announcement and drops, or the reader
// sees "writing x" and excludes that source -- never a torn read.  Readers
// clear the announcement once the call stopped reading the row.  (Flag words
// live in uncached memory: "store -> s_waitcnt vmcnt(0) -> load" is the
// full fence on the GPU, no cache write-back or invalidate involved.)
//
// One call, as roles (GPU: workgroups of one launch; CPU: a progress loop):
//   begin    pick the round (catch-up), announce the gather row
//   push     phase 1: my input's block p -> rank p's SD[row][me], gated
//   decide   per chunk k of my block: wait until floor(thReduce*N) copies
//            landed (or the round is forced), then gate the phase-2 pushes
//   reduce   per piece of chunk k, as soon as k is decided: masked sum ->
//            my output block + every gated peer's GD[row][me]; the last
//            piece of a part stores its "done" tags, the last part marks k
//            reduced (it then counts towards my completion)
//   complete wait until floor(thComplete*total) reduced chunks landed (mine
//            counted once reduced) or the round is forced; publish the set
//   copy     per part of a peer's block: copied to the output as soon as it
//            lands (the reference's per-chunk fire, W:177-181); once the set
//            is published, parts outside it -> 0 (own parts after their
//            reduce pieces); the complete role writes the counts
//   finish   the last workgroup out: withdraw the announcements, publish the
//            call's status, call id + 1
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define OS_HD __host__ __device__
#else
#define OS_HD
#endif

namespace akka {
namespace os {

constexpr int kMaxRanks = 16;
constexpr int kMaxRows = 16;

// ---- tags ---------------------------------------------------------------------
OS_HD inline uint32_t tag_writing(uint32_t r) { return 2u * (r + 1u); }
OS_HD inline uint32_t tag_done(uint32_t r) { return 2u * (r + 1u) + 1u; }
enum TagState : int32_t { kPending = 0, kLanded = 1, kLost = 2 };
// What a tag says about round r's copy.
OS_HD inline int32_t tag_state(uint32_t t, uint32_t r) {
  if (t == tag_done(r)) return kLanded;
  if (t >= tag_writing(r + 1u)) return kLost;  // the single writer moved past round r
  return kPending;
}

// ---- layout of the exported flag area and the local state (uint32 words) -------
struct Layout {
  int32_t N = 0, D = 0, Kmax = 0, P = 0;
  // exported (peers read or write these over the link)
  int64_t stag0 = 0, gtag0 = 0, fired0 = 0, sread0 = 0, gread0 = 0, done0 = 0, seen0 = 0, fin0 = 0, flag_words = 0;
  // local only (this rank's kernels / progress thread)
  int64_t dec0 = 0, okq0 = 0, pctr0 = 0, pdone0 = 0, kctr0 = 0, odone0 = 0, cmask0 = 0, state0 = 0, local_words = 0;

  OS_HD void init(int32_t N_, int32_t D_, int32_t Kmax_, int32_t P_) {
    N = N_;
    D = D_;
    Kmax = Kmax_;
    P = P_;
    const int64_t tags = int64_t(D) * N * Kmax * P;
    stag0 = 0;
    gtag0 = stag0 + 2 * tags;  // (tag, count) pairs
    fired0 = gtag0 + 2 * tags;
    sread0 = fired0 + int64_t(D) * Kmax;
    gread0 = sread0 + int64_t(D) * Kmax;
    done0 = gread0 + D;
    seen0 = done0 + 16;  // its own 64-B line
    fin0 = seen0 + N;
    flag_words = (fin0 + N + 15) / 16 * 16;
    dec0 = 0;  // 64-bit words: even offsets
    okq0 = dec0 + 2 * int64_t(Kmax);
    pctr0 = okq0 + int64_t(Kmax) * P;
    pdone0 = pctr0 + int64_t(Kmax) * P;
    kctr0 = pdone0 + int64_t(Kmax) * P;
    odone0 = kctr0 + Kmax;
    cmask0 = odone0 + Kmax;
    state0 = (cmask0 + int64_t(N) * Kmax + 15) / 16 * 16;
    local_words = state0 + kStateWords;
  }
  // tag word of SD[row][src] chunk k part j (its count word follows)
  OS_HD int64_t stag(int32_t row, int32_t src, int32_t k, int32_t j) const {
    return stag0 + 2 * (((int64_t(row) * N + src) * Kmax + k) * P + j);
  }
  OS_HD int64_t gtag(int32_t row, int32_t blk, int32_t k, int32_t j) const {
    return gtag0 + 2 * (((int64_t(row) * N + blk) * Kmax + k) * P + j);
  }
  OS_HD int64_t fired(int32_t row, int32_t k) const { return fired0 + int64_t(row) * Kmax + k; }
  OS_HD int64_t sread(int32_t row, int32_t k) const { return sread0 + int64_t(row) * Kmax + k; }
  OS_HD int64_t gread(int32_t row) const { return gread0 + row; }
  OS_HD int64_t done() const { return done0; }
  OS_HD int64_t seen(int32_t src) const { return seen0 + src; }
  // src retired: it serves no round >= fin - 1 (0: active)
  OS_HD int64_t fin(int32_t src) const { return fin0 + src; }
  // local: decision of my chunk k, one 64-bit word (landed mask << 32 | round + 1)
  OS_HD int64_t dec(int32_t k) const { return dec0 + 2 * int64_t(k); }
  // local: peers whose gather row takes part j of my chunk k this round (bit q)
  OS_HD int64_t okq(int32_t k, int32_t j) const { return okq0 + int64_t(k) * P + j; }
  // local: finished reduce pieces of part (k, j) / parts of chunk k (counted modulo, never reset)
  OS_HD int64_t pctr(int32_t k, int32_t j) const { return pctr0 + int64_t(k) * P + j; }
  // local: round + 1 once every reduce piece of part (k, j) finished (its output span is final)
  OS_HD int64_t pdone(int32_t k, int32_t j) const { return pdone0 + int64_t(k) * P + j; }
  OS_HD int64_t kctr(int32_t k) const { return kctr0 + k; }
  // local: round + 1 once my chunk k is reduced (self-delivery of its ReduceBlock, W:260-261)
  OS_HD int64_t odone(int32_t k) const { return odone0 + k; }
  // local: chunk (blk, k) is part of this round's output (completion decision)
  OS_HD int64_t cmask(int32_t blk, int32_t k) const { return cmask0 + int64_t(blk) * Kmax + k; }
  OS_HD int64_t state(int32_t i) const { return state0 + i; }

  static constexpr int32_t kStateWords = 16;
};

constexpr int32_t kMaxParts = 64;

// local state words (Layout::state(i))
enum StateWord : int32_t {
  kNext = 0,         // next round this rank may serve
  kCur = 1,          // round of the call in progress
  kCallSeq = 2,      // calls finished on this lane (the next call's id; device-resident)
  kBegun = 3,        // call id + 1 once the call's round is selected
  kCtrFinish = 4,    // workgroups done with the call (the last one out finishes it)
  kCompReason = 5,   // how the completion decision was reached (Verdict)
  kCompLanded = 6,   // chunks landed at the completion decision (mine included)
  kForcedChunks = 7,
  kComp = 8,         // round + 1 once the completion decision (cmask) is published
};

// stats counters (uint64, local device memory / host memory on the CPU)
enum Stat : int32_t {
  kRounds = 0,
  kSkippedRounds,        // rounds jumped over by catch-up at call time
  kScatterPushed,        // (chunk part) pushes that moved bytes
  kScatterOutdated,      // pushes skipped: the owner already reduced that chunk of that round
  kScatterConflict,      // pushes dropped by the overwrite hand-shake
  kGatherPushed,
  kGatherOutdated,       // reduced parts not sent: the receiver already completed the round
  kGatherConflict,
  kReduceThreshold,      // chunk reduces fired at thReduce
  kReduceForced,         // ... forced (catch-up, unreachable, host, timeout)
  kCompleteThreshold,    // rounds completed at thComplete
  kCompleteForced,
  kTimeouts,
  kLandedChunks,         // reduced chunks landed at completion, summed over rounds
  kMissingChunks,
  kDeadSkips,            // pushes not made because the peer is marked dead
  kReduceContribs,       // sum of reduce counts (popcount of the masks)
  kReduceAbandoned,      // my chunks never reduced: the round completed first (W:155-156 drops their scatters)
  kNumStats = 20,
};

// Why a wait ended (0: keep waiting).
enum Verdict : int32_t {
  kWait = 0,
  kThreshold = 1,    // the reference's trigger
  kUnreachable = 2,  // landed + still-possible < needed, and every possible one landed
  kCatchUp = 3,      // a peer pushed a round beyond r + maxLag (W:100-106)
  kHostForce = 4,    // the host forced the round (close / dead peers)
  kTimeout = 5,      // bounded wait expired: forced, and the lane reports an error
  kAbandoned = 6,    // (a chunk's wait only) the round completed first: the chunk is not reduced
};

OS_HD inline int32_t evaluate(int32_t landed, int32_t pending, int32_t need, uint32_t r, int64_t seen_max,
                              int32_t max_lag, uint32_t force_through, bool timed_out) {
  if (landed >= need) return kThreshold;
  // short of the threshold for good (dead or departed peers): still take
  // everything that can arrive before ending the wait -- ending it at once
  // would drop live peers' chunks still in flight
  if (landed + pending < need && pending == 0) return kUnreachable;
  if (seen_max > int64_t(r) + max_lag) return kCatchUp;
  if (force_through > r) return kHostForce;
  if (timed_out) return kTimeout;
  return kWait;
}

// Completion decision (RB:60-66, plus the lane's liveness rules).  My own
// chunks count once reduced (the self-delivered ReduceBlock, W:260-261); a
// FORCED completion (catch-up, unreachable, host force, timeout) first waits
// for every one of them, as the reference force-reduces its own chunks before
// it completes a round (W:101-105) -- they are bounded by their own waits.
OS_HD inline int32_t completion_verdict(int32_t landed_peers, int32_t pending_peers, int32_t own_done, int32_t kme,
                                        int32_t need, uint32_t r, int64_t seen_max, int32_t max_lag,
                                        uint32_t force_through, bool timed_out) {
  const int32_t v = evaluate(landed_peers + own_done, pending_peers + (kme - own_done), need, r, seen_max, max_lag,
                             force_through, timed_out);
  if (v != kWait && v != kThreshold && own_done < kme) return kWait;
  return v;
}

// Round a call serves: the next one, unless a peer already pushed rounds so
// far ahead that it is outside the maxLag window (catch-up skips to the
// oldest round still inside it).
OS_HD inline uint32_t select_round(uint32_t next, int64_t seen_max, int32_t max_lag) {
  const int64_t lo = seen_max - max_lag;
  return lo > int64_t(next) ? uint32_t(lo) : next;
}

// Largest round any peer announced to me (seen words hold round + 1), -1 if none.
template <class M>
OS_HD inline int64_t seen_max(const uint32_t* fl, const Layout& L, int32_t me) {
  int64_t m = -1;
  for (int32_t s = 0; s < L.N; ++s) {
    if (s == me) continue;
    const int64_t v = int64_t(M::ld(fl + L.seen(s))) - 1;
    m = v > m ? v : m;
  }
  return m;
}

// Has source s moved past round r for good?  It announced a later round
// (every push of a rank's round completes before its next round's first
// announcement: one stream, in order) or it retired.  Read this BEFORE the
// tags: a tag read afterwards is then final -- "done r" means landed, anything
// else means s's round-r copy will never come (skipped, dropped or overwritten).
template <class M>
OS_HD inline bool source_past(const uint32_t* fl, const Layout& L, int32_t s, uint32_t r) {
  const uint32_t sn = M::ld(fl + L.seen(s));
  const uint32_t fn = M::ld(fl + L.fin(s));
  return sn > r + 1u || (fn != 0u && r + 1u >= fn);
}

enum Gate : int32_t { kGo = 0, kOutdated = 1, kConflict = 2, kDead = 3 };

// A write dropped by the overwrite hand-shake (kConflict) never happens: its
// "writing r" marker would read as PENDING once the receiver serves round r
// in that row -- a wait only the writer's next round (source_past) or the
// timeout could end, and a writer that stops at r (the end of a job's phase)
// has no next round.  The writer moves the tag to "writing r + 1" instead: a
// round no writer ever writes in this row (D >= 2), read as LOST for round r
// and for every older round, as PENDING for the row's later rounds -- and the
// writer's own later rounds there (r + D, ...) still move the tag forward.
template <class M>
OS_HD inline void retract(uint32_t* tag, uint32_t r) {
  M::st(tag, tag_writing(r + 1u));
}

// Phase 1 sender: may I write round r's part j of chunk k into the owner's
// SD[row][me]?  Leaves the "writing r" marker behind on kGo / kConflict.
template <class M>
OS_HD inline int32_t scatter_gate(uint32_t* owner_fl, const Layout& L, int32_t row, int32_t me, int32_t k, int32_t j,
                                  uint32_t r) {
  if (M::ld(owner_fl + L.fired(row, k)) >= r + 1u) return kOutdated;  // owner reduced round >= r already
  M::st_sc(owner_fl + L.stag(row, me, k, j), tag_writing(r));
  const uint32_t rd = M::ld_sc(owner_fl + L.sread(row, k));
  if (rd != 0u && rd != r + 1u) {  // owner is reading this row for another round
    retract<M>(owner_fl + L.stag(row, me, k, j), r);
    return kConflict;
  }
  return kGo;
}

// Phase 2 sender (block owner `me`): may I write my reduced part into
// receiver q's GD[row][me]?
template <class M>
OS_HD inline int32_t gather_gate(uint32_t* q_fl, const Layout& L, int32_t row, int32_t me, int32_t k, int32_t j,
                                 uint32_t r) {
  if (M::ld(q_fl + L.done()) >= r + 1u) return kOutdated;  // q completed round >= r already
  M::st_sc(q_fl + L.gtag(row, me, k, j), tag_writing(r));
  const uint32_t rd = M::ld_sc(q_fl + L.gread(row));
  if (rd != 0u && rd != r + 1u) {
    retract<M>(q_fl + L.gtag(row, me, k, j), r);
    return kConflict;
  }
  // q may have completed round r between the first look and the marker:
  // look again AFTER the marker (q stores done, then reads the tags it
  // zeroes under), so either this write drops or q sees "writing r" and
  // waits for it before zeroing -- with the window output the row IS the
  // caller's result, and a late write must not land on top of its zeros
  if (M::ld_sc(q_fl + L.done()) >= r + 1u) {
    retract<M>(q_fl + L.gtag(row, me, k, j), r);
    return kOutdated;
  }
  return kGo;
}

// A tag of gather row `row` that says a writer may still be storing into the
// row: "writing y" for a round y that lives in this row.  A retracted marker
// ("writing x + 1" after x's write dropped, x in this row) names a round of
// the NEXT row (D >= 2), so it never reads as in flight.
OS_HD inline bool writer_in_flight(uint32_t t, int32_t row, int32_t D) {
  return t != 0u && (t & 1u) == 0u && int32_t((t / 2u - 1u) % uint32_t(D)) == row;
}

// Host-visible per-call status record (host memory, written by the last
// workgroup of the call's final kernel).  Slot = call id % kStatusSlots; the
// record names its call, so a reader holding an older call's slot sees that
// the slot was reused instead of another call's round.
struct CallStatus {
  int64_t call;           // call id (lane's call sequence number)
  int64_t round;          // round served (-1 until the call finished)
  int64_t reason;         // completion Verdict
  int64_t landed_chunks;  // reduced chunks landed at completion (mine included)
  int64_t forced_chunks;  // my chunks whose reduce was forced
  int64_t pad[3];
};
constexpr int kStatusSlots = 64;

}  // namespace os
}  // namespace akka
