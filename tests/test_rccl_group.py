"""The gate's grouped communicator init (``ops/csrc/tk_rccl_group.h``) against a mock RCCL.

``tk_rccl_probe.hip`` brings up a node's share of the cluster communicator with one
``ncclCommInitRank`` per local GPU inside one group.  On a one-GPU pool that path with
``ndev > 1`` never runs, so the first 8-GPU node would be its first execution.  The
sequence is a host-only template; here it is compiled with the host compiler against a
mock that enforces RCCL's contract (every violation is an error the mock reports):

* all of a process's inits inside ONE ``ncclGroupStart``/``ncclGroupEnd``, balanced even
  after a failure;
* the current device set to rank d's GPU right before rank d's init;
* no GPU twice in one process, ranks in ``[0, world)`` and never claimed twice, one world
  size per unique id.

Shapes: one process with 8 GPUs (world 8); 8 processes with 8 GPUs each (world 64); a
``hipSetDevice`` failure and an init failure mid-group; bad geometries.
"""

import json
import shutil
import subprocess

import pytest

from test_rccl_verify import CSRC

DRIVER = r"""
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <vector>
#include "tk_rccl_group.h"

// the "bootstrap": what every process of a world registered under one unique id
struct Registry {
  int world = -1;
  std::set<int> ranks;
  std::vector<std::string> violations;
};

struct MockApi {
  using Comm = int;
  static constexpr int kInvalidArgument = 4;
  Registry* reg;
  int visible = 8;
  int fail_set_device_at = -1, fail_init_at = -1;
  // process state
  int depth = 0, starts = 0, ends = 0, current = -1, inits = 0, sets = 0;
  bool device_fresh = false;  // set_device since the last init
  std::set<int> bound;        // GPUs holding a rank of this communicator in this process
  std::vector<std::string>& v() { return reg->violations; }
  int group_start() { ++starts; if (depth++) v().push_back("nested ncclGroupStart"); return 0; }
  int group_end() { ++ends; if (--depth) v().push_back("unbalanced ncclGroupEnd"); return 0; }
  int set_device(int dev) {
    if (sets++ == fail_set_device_at) return 1;
    if (dev < 0 || dev >= visible) { v().push_back("hipSetDevice out of range"); return 1; }
    current = dev; device_fresh = true; return 0;
  }
  int init_rank(Comm* c, int world, int rank) {
    if (inits == fail_init_at) { ++inits; return 3; }
    ++inits;
    if (depth != 1) v().push_back("ncclCommInitRank outside the group");
    if (!device_fresh) v().push_back("ncclCommInitRank without hipSetDevice before it");
    device_fresh = false;
    if (!bound.insert(current).second) v().push_back("two ranks on GPU " + std::to_string(current));
    if (reg->world < 0) reg->world = world;
    if (reg->world != world) v().push_back("one unique id, two world sizes");
    if (rank < 0 || rank >= world) v().push_back("rank out of range");
    if (!reg->ranks.insert(rank).second) v().push_back("rank " + std::to_string(rank) + " claimed twice");
    *c = rank;
    return 0;
  }
  const char* error_string(int r) { return r == 3 ? "mock internal error" : "mock invalid argument"; }
};

static void run(const char* name, int nproc, int ndev, int world, int fail_set, int fail_init) {
  Registry reg;
  std::vector<int> rcs;
  std::string errs;
  int starts = 0, ends = 0;
  for (int p = 0; p < nproc; ++p) {
    MockApi api{&reg};
    api.fail_set_device_at = p == 0 ? fail_set : -1;
    api.fail_init_at = p == 0 ? fail_init : -1;
    std::vector<int> devs(ndev), comms(ndev, -1);
    for (int d = 0; d < ndev; ++d) devs[d] = d;  // every node's own GPUs 0..ndev-1
    char err[256] = {0};
    rcs.push_back(tk_group_init(api, world, p * ndev, ndev, devs.data(), comms.data(), err, sizeof(err)));
    if (err[0]) errs += std::string(err) + ";";
    starts += api.starts; ends += api.ends;
  }
  std::printf("{\"case\":\"%s\",\"rcs\":[", name);
  for (size_t i = 0; i < rcs.size(); ++i) std::printf("%s%d", i ? "," : "", rcs[i]);
  std::printf("],\"ranks\":%zu,\"starts\":%d,\"ends\":%d,\"errors\":\"%s\",\"violations\":[", reg.ranks.size(),
              starts, ends, errs.c_str());
  for (size_t i = 0; i < reg.violations.size(); ++i) std::printf("%s\"%s\"", i ? "," : "", reg.violations[i].c_str());
  std::printf("]}\n");
}

static void geometry(const char* name, int world, int rank_base, std::vector<int> devs) {
  char err[256] = {0};
  const int rc = tk_check_geometry(world, rank_base, (int)devs.size(), devs.data(), err, sizeof(err));
  std::printf("{\"case\":\"%s\",\"rc\":%d,\"error\":\"%s\"}\n", name, rc, err);
}

int main() {
  run("node8", 1, 8, 8, -1, -1);
  run("cluster64", 8, 8, 64, -1, -1);
  run("set_device_fails", 1, 8, 8, 3, -1);
  run("init_fails", 1, 8, 8, -1, 5);
  geometry("ok", 64, 56, {0, 1, 2, 3, 4, 5, 6, 7});
  geometry("dup", 16, 0, {0, 1, 1, 3});
  geometry("past_world", 8, 4, {0, 1, 2, 3, 4, 5});
  geometry("negative", 8, 0, {0, -1});
  return 0;
}
"""


@pytest.fixture(scope="module")
def cases(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("group")
    (d / "main.cpp").write_text(DRIVER)
    subprocess.run([cxx, "-std=c++17", "-O1", "-Wall", "-Werror", "-I", CSRC, str(d / "main.cpp"), "-o",
                    str(d / "mock")], check=True)
    out = subprocess.run([str(d / "mock")], capture_output=True, text=True, check=True).stdout
    return {c["case"]: c for c in map(json.loads, out.splitlines())}


def test_one_node_of_eight_gpus(cases):
    c = cases["node8"]
    assert c["rcs"] == [0] and c["ranks"] == 8 and c["violations"] == []
    assert (c["starts"], c["ends"]) == (1, 1)  # one group per process


def test_eight_nodes_of_eight_gpus(cases):
    c = cases["cluster64"]
    assert c["rcs"] == [0] * 8 and c["ranks"] == 64 and c["violations"] == []
    assert (c["starts"], c["ends"]) == (8, 8)


def test_failure_inside_the_group_still_ends_it(cases):
    for name, msg in (("set_device_fails", "hipSetDevice(3) failed"), ("init_fails", "mock internal error")):
        c = cases[name]
        assert c["rcs"][0] != 0 and msg in c["errors"], c
        assert (c["starts"], c["ends"]) == (1, 1) and c["violations"] == []


def test_geometry(cases):
    assert cases["ok"]["rc"] == 0
    assert "device 1 given to ranks 1 and 2 of one process" in cases["dup"]["error"]
    assert "world=8 rank_base=4 ndev=6" in cases["past_world"]["error"]
    assert cases["negative"]["rc"] == -1


def test_the_probe_uses_the_tested_sequence():
    src = open(f"{CSRC}/tk_rccl_probe.hip").read()
    assert "tk_group_init(api, g->world, g->rank_base" in src
    assert "if (tk_check_geometry(world, rank_base, ndev, devices, g_err, sizeof(g_err))) return -1;" in src
    assert src.count("ncclCommInitRank(") == 1  # the adapter's, called only through tk_group_init
