"""The RCCL gate's verification rule (``ops/csrc/tk_rccl_verify.h``) on the CPU.

The gate compares the all-reduced buffer with the exact sum, so every partial sum the
collective forms must be representable in the wire type.  Round 3 used ``rank + 1`` for
every world, which is exact in bf16 only up to 15 ranks: a 64-rank bf16 gate reported
corruption that was rounding.  Here the header is compiled with the host compiler and its
values are pushed through a simulation of the reduction in bf16 (``torch.bfloat16``
rounding after every add) in ring order and in tree order, for every world up to 256;
above 256 bf16 is refused, by the library and by ``rccl-ready --bf16`` before any
communicator exists.
"""

import os
import shutil
import subprocess

import pytest
import torch

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "triton_kubernetes_amd", "ops",
                    "csrc")

DRIVER = r"""
#include <cstdio>
#include "tk_rccl_verify.h"
int main() {
  for (int dtype = 0; dtype < 2; ++dtype)
    for (int world = 1; world <= 300; ++world) {
      std::printf("%d %d %d %.1f", dtype, world, tk_verifiable(dtype, world) ? 1 : 0, tk_verify_sum(dtype, world));
      for (int r = 0; r < world; ++r) std::printf(" %.1f", tk_verify_value(dtype, world, r));
      std::printf("\n");
    }
  return 0;
}
"""


@pytest.fixture(scope="module")
def rule(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("c++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    d = tmp_path_factory.mktemp("verify")
    (d / "main.cpp").write_text(DRIVER)
    subprocess.run([cxx, "-std=c++17", "-O1", "-I", CSRC, str(d / "main.cpp"), "-o", str(d / "rule")], check=True)
    out = {}
    for line in subprocess.run([str(d / "rule")], capture_output=True, text=True, check=True).stdout.splitlines():
        f = line.split()
        out[(int(f[0]), int(f[1]))] = (f[2] == "1", float(f[3]), [float(x) for x in f[4:]])
    return out


def _bf16_add(a, b):
    return (torch.tensor(a, dtype=torch.bfloat16) + torch.tensor(b, dtype=torch.bfloat16)).item()


def _ring(values):
    """Ring reduce-scatter: the chunk owned by rank k accumulates ranks k+1, k+2, ... in
    turn, rounding after every hop (all-gather then copies it unchanged)."""
    n = len(values)
    results = set()
    for start in range(min(n, 8)):
        acc = torch.tensor(values[start], dtype=torch.bfloat16).item()
        for hop in range(1, n):
            acc = _bf16_add(acc, values[(start + hop) % n])
        results.add(acc)
    return results


def _tree(values):
    layer = [torch.tensor(v, dtype=torch.bfloat16).item() for v in values]
    while len(layer) > 1:
        nxt = [_bf16_add(layer[i], layer[i + 1]) for i in range(0, len(layer) - 1, 2)]
        if len(layer) % 2:
            nxt.append(layer[-1])
        layer = nxt
    return layer[0]


def test_f32_rule_is_rank_plus_one(rule):
    for world in (1, 2, 8, 64, 256):
        ok, want, vals = rule[(0, world)]
        assert ok and vals == [float(r + 1) for r in range(world)] and want == world * (world + 1) / 2


@pytest.mark.parametrize("world", [2, 8, 15, 16, 17, 64, 100, 128, 200, 255, 256])
def test_bf16_partial_sums_are_exact_in_every_order(rule, world):
    ok, want, vals = rule[(1, world)]
    assert ok
    assert _ring(vals) == {want}
    assert _tree(vals) == want


def test_round3_rule_was_wrong_past_15_ranks():
    """What the gate used before: rank + 1 in bf16 rounds away from the exact sum."""
    vals = [float(r + 1) for r in range(64)]
    assert _tree(vals) != 64 * 65 / 2 or _ring(vals) != {64 * 65 / 2}


def test_bf16_refused_above_256_ranks(rule):
    assert rule[(1, 256)][0] and not rule[(1, 257)][0] and rule[(0, 300)][0]
    src = open(os.path.join(CSRC, "tk_rccl_probe.hip")).read()
    # the library refuses in the sweep, the executable before any communicator exists
    assert "rc = check_verifiable(dtype, g->world);" in src
    assert "if (check_verifiable(dtype, world)) {  // refused before any communicator exists" in src
    from triton_kubernetes_amd.ops import rccl

    with pytest.raises(ValueError, match="at most 256 ranks"):
        rccl.check_dtype("bf16", 257)
    rccl.check_dtype("bf16", 256)
    rccl.check_dtype("f32", 4096)
