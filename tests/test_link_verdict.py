"""The xGMI link-check verdict exists twice: ``gpu-burnin --p2p`` on SSH / Terraform nodes
(``ops/csrc/tk_link_verdict.h``) and the node agent (``node/labels.py:link_labels`` and
``best_link_verdict``'s retry rule).  Property test: both judge generated matrices alike --
status, degraded / below-floor / corrupt counts, min and median, and whether the matrix is
worth measuring again.  The C++ side runs in a small host-only harness built here with g++."""

import json
import os
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from triton_kubernetes_amd.node.labels import link_labels

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "triton_kubernetes_amd", "ops", "csrc")
HARNESS = r'''
#include <cstdio>
#include <vector>
#include "tk_link_verdict.h"
int main() {
  int n; double frac, floor_;
  while (scanf("%d %lf %lf", &n, &frac, &floor_) == 3) {
    std::vector<double> mat(n * n), derr(n * n);
    std::vector<int> acc(n * n);
    for (auto& x : mat) if (scanf("%lf", &x) != 1) return 1;
    for (auto& x : acc) if (scanf("%d", &x) != 1) return 1;
    for (auto& x : derr) if (scanf("%lf", &x) != 1) return 1;
    const TkLinkVerdict v = tk_link_verdict(n, mat.data(), acc.data(), derr.data(), frac, floor_);
    printf("{\"status\":\"%s\",\"degraded\":%d,\"below_floor\":%d,\"corrupt\":%d,\"min\":%.1f,\"median\":%.2f,"
           "\"slow_only\":%d}\n", v.status, v.degraded, v.below_floor, v.corrupt, v.min_gbps, v.median_gbps,
           (int)tk_link_slow_only(n, mat.data(), acc.data(), derr.data(), frac, floor_));
  }
  return 0;
}
'''


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("linkv")
    src, exe = d / "h.cpp", d / "h"
    src.write_text(HARNESS)
    # under ASan + UBSan: the verdict reads n*n arrays the harness sizes from its input
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-Wall", "-Werror", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-I", CSRC, str(src), "-o", str(exe)], check=True)
    return str(exe)


def _cpp(exe, cases):
    text = ""
    for n, frac, floor_, mat, acc, derr in cases:
        text += f"{n} {frac} {floor_}\n" + " ".join(map(str, mat)) + "\n" + " ".join(map(str, acc)) + "\n" + \
            " ".join(map(str, derr)) + "\n"
    out = subprocess.run([exe], input=text, capture_output=True, text=True, check=True).stdout
    return [json.loads(line) for line in out.splitlines()]


def _python(n, frac, floor_, mat, acc, derr):
    """The matrix as ops/probe.py:link_matrix reports it, judged by node/labels.py."""
    pairs, access, errors, data = {}, {}, [], {}
    for i in range(n):
        for j in range(n):
            if i == j:
                continue
            v = mat[i * n + j]
            access[f"{i}-{j}"] = bool(acc[i * n + j])
            if v < 0:
                errors.append(f"{i}->{j}: peer read failed")
                continue
            pairs[f"{i}-{j}"] = v
            if derr[i * n + j] > 0:
                data[f"{i}-{j}"] = int(derr[i * n + j])
    got = link_labels({"pairs": pairs, "peer_access": access, "errors": errors, "data_errors": data}, frac, floor_)
    lab = got["labels"]
    return {"status": got["status"], "degraded": len(got["degraded"]), "below_floor": len(got["below_floor"]),
            "corrupt": len(got.get("corrupt", [])), "min": float(lab.get("amd.com/xgmi.p2p-min-gbps", 0)) if pairs else 0.0,
            "median": float(lab.get("amd.com/xgmi.p2p-median-gbps", 0)) if pairs else 0.0,
            # best_link_verdict measures again while the verdict is degraded for speed alone
            "slow_only": int(got["status"] == "degraded" and not got.get("corrupt"))}


@st.composite
def matrices(draw):
    n = draw(st.integers(2, 8))
    nn = n * n
    # GB/s at the 0.1 resolution ops/probe.py reports; mostly healthy, some slow, a few failed
    val = st.one_of(st.integers(450, 650), st.integers(0, 450), st.just(-10)).map(lambda x: x / 10.0)
    mat = draw(st.lists(val, min_size=nn, max_size=nn))
    acc = draw(st.lists(st.sampled_from([1, 1, 1, 1, 0]), min_size=nn, max_size=nn))
    derr = draw(st.lists(st.sampled_from([0, 0, 0, 0, 0, 0, 3]), min_size=nn, max_size=nn))
    frac = draw(st.sampled_from([0.5, 0.75]))
    floor_ = draw(st.sampled_from([0.0, 38.0, 45.0]))
    return n, frac, floor_, mat, acc, derr


@settings(max_examples=150, deadline=None)
@given(st.lists(matrices(), min_size=1, max_size=20))
def test_cpp_and_python_verdicts_agree(harness, cases):
    for case, cpp in zip(cases, _cpp(harness, cases)):
        py = _python(*case)
        # the labels carry min / median rounded to whole GB/s
        assert cpp["status"] == py["status"], (case, cpp, py)
        assert (cpp["degraded"], cpp["below_floor"], cpp["corrupt"], cpp["slow_only"]) == \
            (py["degraded"], py["below_floor"], py["corrupt"], py["slow_only"]), (case, cpp, py)
        if py["min"] or py["median"]:
            assert round(cpp["min"]) == py["min"] and round(cpp["median"]) == py["median"], (case, cpp, py)


def test_known_cases(harness):
    healthy = [0 if i == j else 60.0 for i in range(4) for j in range(4)]
    slow = list(healthy)
    slow[1] = 20.0  # 0 -> 1 at a third of the median
    corrupt = [0.0] * 16
    corrupt[6] = 5
    ones = [1] * 16
    cases = [(4, 0.5, 38.0, healthy, ones, [0.0] * 16), (4, 0.5, 38.0, slow, ones, [0.0] * 16),
             (4, 0.5, 38.0, healthy, ones, corrupt), (4, 0.5, 70.0, healthy, ones, [0.0] * 16)]
    got = _cpp(harness, cases)
    assert [g["status"] for g in got] == ["passed", "degraded", "degraded", "degraded"]
    assert [g["slow_only"] for g in got] == [0, 1, 0, 1]  # wrong data is never measured away
    assert got[3]["below_floor"] == 12
