// Phase watchdog: a native thread that ends the process legibly when a phase
// of a multi-rank job overruns its deadline (or the launcher sends SIGTERM).
//
// Why native: the calls that hang on a missing peer (ncclCommInitRank, the
// first ncclGroupEnd that connects a p2p channel, a stream synchronize behind
// a p2p kernel) sit inside C with the Python GIL held, so a Python timer could
// never run.  This thread needs neither the GIL nor the HIP runtime: it waits
// on a pipe with a deadline, and on expiry writes the pre-composed failure
// line (with the tail of this rank's RCCL debug log spliced in) and _exit()s.
//
// The reference has nothing comparable: a lost Akka member is declared down by
// the cluster failure detector after 10 s (application.conf:18-20) and the
// master just stops counting it (AllreduceMaster.scala:46-52).
#pragma once

#include <string>

namespace akka {

// Arm (or re-arm) the watchdog.  `line` is written on expiry, to stdout when
// `to_stdout`, else to stderr; the JSON string tokens "__AKKA_REASON__" and
// "__AKKA_TAIL__" (quotes included) are replaced by JSON strings holding the
// reason and the last `tail_bytes` of `debug_path` (if readable).
// `beacon_path` (optional): a file any rank creates when it fails; while
// armed, the watchdog checks for it every 200 ms and fires at once ("failure
// reported by a rank: <file contents>"), so one rank's error ends every rank promptly
// even when the others are blocked in a collective that will never match.
// The descriptor failure lines go to when `to_stdout` (default 1): a program
// that moves fd 1 elsewhere keeps a private copy of its real stdout here.
void watchdog_set_out_fd(int fd);
void watchdog_arm(double seconds, const std::string& line, bool to_stdout, const std::string& debug_path,
                  int exit_code, int tail_bytes, const std::string& beacon_path = "");
void watchdog_disarm();
// Route SIGTERM through the watchdog: the armed line is written (reason
// "SIGTERM") before the process exits; unarmed, it exits with 128+15.
void watchdog_install_sigterm();
// Child processes killed (SIGKILL) when the watchdog ends this process
// (deadline, beacon or SIGTERM).  At most 16; false when the table is full.
bool watchdog_track_child(int pid);
void watchdog_untrack_child(int pid);
// Expose the escaping used for the tail (tests).
std::string json_escape(const std::string& s);

}  // namespace akka
