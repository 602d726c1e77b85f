// A gate's communicator bring-up in one process (tk_rccl_probe.hip): its geometry and the
// grouped ncclCommInitRank sequence, as host-only templates so the contract with RCCL is
// unit-tested on the CPU against a mock that enforces it (tests/test_rccl_group.py) -- the
// 8-GPU path runs for the first time on an 8-GPU node, and must not fail there on a
// sequencing mistake a CPU test can see.
//
// RCCL's contract for one process joining a communicator with several GPUs:
//  * ranks rank_base .. rank_base+ndev-1 lie in [0, world), and every process of the world
//    uses the same unique id with the same world size;
//  * no two ranks of one communicator on one GPU in one process ("Duplicate GPU detected");
//  * all of the process's ncclCommInitRank calls inside ONE ncclGroupStart/ncclGroupEnd
//    (otherwise the first call blocks waiting for ranks this same thread would init next);
//  * before rank d's ncclCommInitRank the current device is rank d's GPU (the communicator
//    binds to the current device);
//  * ncclGroupEnd is called even when a call inside the group failed.
#pragma once

#include <cstddef>
#include <cstdio>

// 0, or -1 with `err` set.
static inline int tk_check_geometry(int world, int rank_base, int ndev, const int* devices, char* err,
                                    size_t errlen) {
  if (ndev < 1 || world < ndev || rank_base < 0 || rank_base + ndev > world) {
    snprintf(err, errlen, "bad gate geometry: world=%d rank_base=%d ndev=%d", world, rank_base, ndev);
    return -1;
  }
  for (int a = 0; a < ndev; ++a) {
    if (devices[a] < 0) {
      snprintf(err, errlen, "bad gate geometry: device %d", devices[a]);
      return -1;
    }
    for (int b = a + 1; b < ndev; ++b)
      if (devices[a] == devices[b]) {
        snprintf(err, errlen, "bad gate geometry: device %d given to ranks %d and %d of one process", devices[a],
                 rank_base + a, rank_base + b);
        return -1;
      }
  }
  return 0;
}

// Api: group_start() / group_end() / init_rank(Comm*, world, rank) -> 0 or an error code;
// set_device(dev) -> 0 or non-zero; error_string(code).  Returns 0 or the first error code,
// with `err` set.
template <class Api>
int tk_group_init(Api& api, int world, int rank_base, int ndev, const int* devices, typename Api::Comm* comms,
                  char* err, size_t errlen) {
  int r = api.group_start();
  for (int d = 0; d < ndev && r == 0; ++d) {
    if (api.set_device(devices[d]) != 0) {
      snprintf(err, errlen, "hipSetDevice(%d) failed", devices[d]);
      r = Api::kInvalidArgument;
      break;
    }
    r = api.init_rank(&comms[d], world, rank_base + d);
  }
  const int re = api.group_end();  // balanced even after a failure inside the group
  if (r == 0) r = re;
  if (r != 0 && !err[0]) snprintf(err, errlen, "ncclCommInitRank: %s", api.error_string(r));
  return r;
}
