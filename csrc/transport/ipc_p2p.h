// Host-side planning of one IpcP2P group (ipc_p2p.cpp), separate from the
// device so it can be checked on a CPU: ops grouped into queues per
// (direction, peer, channel) in issue order, each op given the sequence
// number of its first mailbox piece.
#pragma once

#include <cstdint>
#include <vector>

#include "../kernels/ipc_kernels.h"
#include "p2p.h"

namespace akka {

struct IpcP2PPlan {
  std::vector<IpcP2POp> ops;    // queue by queue, issue order inside a queue
  std::vector<int32_t> qstart;  // [nqueues + 1]
  int64_t bytes_sent = 0;
};

// `dead[p]` != 0: transfers with p are dropped.  `send_seq` / `recv_seq`
// ([peer * nch + ch], next piece number) advance by the pieces planned.
IpcP2PPlan plan_ipc_p2p_group(const std::vector<P2POp>& ops, int32_t nranks, int64_t piece, int32_t nch,
                              const uint32_t* dead, std::vector<uint32_t>& send_seq, std::vector<uint32_t>& recv_seq);

}  // namespace akka
