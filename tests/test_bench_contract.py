"""The headline bench times the product's defaults, and never a previous step's HBM release.

* ``bench.py``'s burn-in level defaults to ``models/baremetal.DEFAULT_BURNIN`` (VERDICT r4
  "Next round" #3): the line's ``config.burnin`` is the level a node ships with.
* ``ops/hbm.settle`` (the untimed wait between steps) returns once the driver's VRAM
  clearing backlog, as ``mem_info_vram_used`` shows it, has drained.
"""

import os
import sys
import threading
import time

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from triton_kubernetes_amd.models.baremetal import DEFAULT_BURNIN  # noqa: E402
from triton_kubernetes_amd.ops import hbm  # noqa: E402


def test_bench_burnin_default_is_the_product_default(monkeypatch):
    import bench

    monkeypatch.setattr(sys, "argv", ["bench.py"])
    args = bench.parse_args()
    assert args.burnin == DEFAULT_BURNIN == "full"
    assert args.hbm_settle == "on"


def test_smoke_stays_on_the_explicit_quick_level():
    import __graft_entry__ as entry
    import inspect

    src = inspect.getsource(entry.smoke)
    assert '"--burnin", "quick"' in src


def _card(root, name, used):
    d = os.path.join(root, name, "device")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "mem_info_vram_used"), "w") as fh:
        fh.write(f"{used}\n")
    return os.path.join(d, "mem_info_vram_used")


def test_vram_used_reads_cards_not_connectors(tmp_path):
    _card(str(tmp_path), "card0", 5 << 30)
    _card(str(tmp_path), "card1", 7 << 30)
    os.makedirs(tmp_path / "card0-DP-1" / "device")
    (tmp_path / "card0-DP-1" / "device" / "mem_info_vram_used").write_text("123\n")
    assert hbm.vram_used(str(tmp_path)) == {"card0": 5 << 30, "card1": 7 << 30}


def test_settle_without_amdgpu_returns_at_once(tmp_path):
    got = hbm.settle(str(tmp_path))
    assert got["cards"] == 0 and got["waited_s"] == 0.0


def test_settle_waits_for_the_backlog_to_drain(tmp_path):
    """A card releasing 40 GiB at 1 GiB per 10 ms: settle returns after the drain, not before."""
    path = _card(str(tmp_path), "card0", 48 << 30)
    done = threading.Event()

    def drain():
        used = 48 << 30
        while used > (8 << 30):
            time.sleep(0.01)
            used -= 1 << 30
            with open(path + ".tmp", "w") as fh:
                fh.write(f"{used}\n")
            os.replace(path + ".tmp", path)
        done.set()

    t = threading.Thread(target=drain)
    t.start()
    # a quiet window 50x the drain's step: a loaded test host (pytest -n 8) can stall the
    # drain thread for a while, and a stall longer than the window reads as "drained"
    got = hbm.settle(str(tmp_path), quiet_s=0.5, poll_s=0.005, timeout_s=20)
    t.join()
    assert done.is_set()
    assert got["released_gib"] == pytest.approx(40, abs=1.5)
    assert not got["timed_out"]


def test_settle_floor_exits_early(tmp_path):
    _card(str(tmp_path), "card0", 8 << 30)
    t0 = time.monotonic()
    got = hbm.settle(str(tmp_path), quiet_s=5.0, floor=8 << 30)
    assert time.monotonic() - t0 < 1.0 and not got["timed_out"] and got["reached_floor"]


def test_settle_waits_for_a_release_that_has_not_started(tmp_path):
    """An exited process's memory comes back later (the driver's deferred teardown): with a
    floor the wait holds on until the level is back, not just for a quiet window."""
    path = _card(str(tmp_path), "card0", 40 << 30)

    def later():
        time.sleep(0.6)  # nothing for longer than the quiet window, then the release
        for used in (24 << 30, 8 << 30, 1 << 30):
            with open(path + ".tmp", "w") as fh:
                fh.write(f"{used}\n")
            os.replace(path + ".tmp", path)
            time.sleep(0.05)

    t = threading.Thread(target=later)
    t.start()
    got = hbm.settle(str(tmp_path), quiet_s=1.0, poll_s=0.005, timeout_s=10, floor=1 << 30, slack=0)
    t.join()
    assert got["reached_floor"] and got["waited_s"] >= 0.6 and got["floor"] == 1 << 30


def test_settle_times_out_on_a_card_that_keeps_falling(tmp_path):
    path = _card(str(tmp_path), "card0", 1 << 40)
    stop = threading.Event()

    def fall():
        used = 1 << 40
        while not stop.is_set():
            used -= 1 << 20
            with open(path + ".tmp", "w") as fh:
                fh.write(f"{used}\n")
            os.replace(path + ".tmp", path)
            time.sleep(0.002)

    t = threading.Thread(target=fall)
    t.start()
    try:
        got = hbm.settle(str(tmp_path), quiet_s=0.4, poll_s=0.005, timeout_s=1.0)
    finally:
        stop.set()
        t.join()
    assert got["timed_out"]


def test_cards_for_pci_picks_this_process_gpus(tmp_path):
    """A shared host lists every tenant's GPU: only the cards at our PCI addresses count."""
    for card, bdf, used in (("card0", "0000:05:00.0", 1 << 30), ("card8", "0000:75:00.0", 200 << 30),
                            ("card16", "0001:e5:00.0", 9 << 30)):
        pci = tmp_path / "pci" / bdf
        pci.mkdir(parents=True)
        (pci / "mem_info_vram_used").write_text(f"{used}\n")
        (tmp_path / "drm" / card).mkdir(parents=True)
        os.symlink(pci, tmp_path / "drm" / card / "device")
    drm = str(tmp_path / "drm")
    assert hbm.cards_for_pci([(0, 0x75, 0)], drm) == ["card8"]
    assert hbm.cards_for_pci([(1, 0xE5, 0), (0, 5, 0)], drm) == ["card0", "card16"]
    assert hbm.vram_used(drm, cards=["card8"]) == {"card8": 200 << 30}
    assert hbm.cards_for_pci([(0, 0x99, 0)], drm) == []
    assert hbm.settle(drm, cards=[])["cards"] == 0


def test_comgr_cache_dir_follows_comgr_own_lookup(monkeypatch, tmp_path):
    """The line reports the code-object cache the timed steps find (node state the warmup
    fills): comgr's own directory choice, explicit dir first, then XDG, then ~/.cache."""
    import bench

    monkeypatch.setenv("AMD_COMGR_CACHE_DIR", str(tmp_path / "x"))
    assert bench.comgr_cache_dir() == str(tmp_path / "x")
    monkeypatch.delenv("AMD_COMGR_CACHE_DIR")
    monkeypatch.setenv("XDG_CACHE_HOME", str(tmp_path / "xdg"))
    assert bench.comgr_cache_dir() == str(tmp_path / "xdg" / "comgr")
    monkeypatch.delenv("XDG_CACHE_HOME")
    monkeypatch.setenv("HOME", str(tmp_path / "home"))
    assert bench.comgr_cache_dir() == str(tmp_path / "home" / ".cache" / "comgr")
    (tmp_path / "home" / ".cache" / "comgr").mkdir(parents=True)
    (tmp_path / "home" / ".cache" / "comgr" / "entry").write_bytes(b"\0" * (3 << 20))
    assert bench.dir_mib(bench.comgr_cache_dir()) == 3.0


def test_agent_unit_gives_comgr_a_cache_dir():
    import os

    from triton_kubernetes_amd.images import packer

    unit = open(os.path.join(packer.FILES_DIR, "tk-node-agent.service")).read()
    assert "Environment=AMD_COMGR_CACHE_DIR=/var/cache/triton-kubernetes/comgr" in unit
    assert "CacheDirectory=triton-kubernetes/comgr" in unit


def test_prewarm_is_one_device_code_load_in_a_throwaway_process():
    """A fresh box's cold code-object cache is filled before the timed region, the way a
    booted node's agent fills it: one preload of RCCL's device code, nothing else."""
    import bench

    code = bench._prewarm_code()
    compile(code, "<prewarm>", "exec")
    assert "rccl.preload_device_code([0])" in code and "GateComm" not in code
    assert bench.COMGR_WARM_MIB < 540  # librccl's unbundled gfx950 code, once cached


def test_resident_settles_learn_the_resident_floor():
    """Warm creates keep their agents up: the first settle cannot reach the cold floor and
    ends on its quiet window; its end level becomes the floor the later settles stop at."""
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)

    class FakeHBM:
        def __init__(self):
            self.used, self.calls = 5 << 30, []

        def settle(self, cards, floor):
            self.calls.append(floor)
            reached = floor is not None and self.used <= floor["card0"] + (1 << 30)
            return {"waited_s": 0.1, "floor_by_card": {"card0": min(self.used, floor["card0"]) if floor else self.used},
                    "reached_floor": reached, "timed_out": False}

        def vram_used(self, cards):
            return {c: self.used // len(cards) for c in cards}

    hbm = FakeHBM()
    cold = [None]
    bench.settle_cards(hbm, ["card0"], cold, resident=False)
    assert cold == [{"card0": 5 << 30}]
    hbm.used = 9 << 30  # resident agents up: 4 GiB of their own
    warm = [None]
    first = bench.settle_cards(hbm, ["card0"], warm, resident=True)
    assert not first["reached_floor"] and warm == [{"card0": 9 << 30}]
    again = bench.settle_cards(hbm, ["card0"], warm, resident=True)
    assert again["reached_floor"] and hbm.calls == [None, None, {"card0": 9 << 30}] and cold == [{"card0": 5 << 30}]


def test_settle_slack_is_per_card(tmp_path):
    """The floor is a sum over the node's cards: each card may sit a little above its own
    clean level, so the default slack is 1 GiB per card (8 cards: 8 GiB), not 1 GiB in all."""
    for i in range(8):
        _card(str(tmp_path), f"card{i}", (1 << 30) + (900 << 20))  # 900 MiB above a 1 GiB floor each
    got = hbm.settle(str(tmp_path), quiet_s=5.0, poll_s=0.005, timeout_s=10, floor=8 << 30)
    assert got["reached_floor"] and got["waited_s"] < 1.0
    got = hbm.settle(str(tmp_path), quiet_s=0.2, poll_s=0.005, timeout_s=10, floor=8 << 30, slack=1 << 30)
    assert not got["reached_floor"]


def test_settle_per_card_floor_waits_for_the_card_still_clearing(tmp_path):
    """Per-card floors: seven idle cards at their level do not end the wait while the eighth
    still has most of a burn-in's release to clear (a summed floor with 8 GiB of slack
    would have let ~7 GiB of clearing run into the next step)."""
    paths = [_card(str(tmp_path), f"card{i}", 1 << 30) for i in range(8)]
    with open(paths[3], "w") as fh:
        fh.write(f"{(1 << 30) + (7 << 30)}\n")  # 7 GiB left to clear on card3
    floor = {f"card{i}": 1 << 30 for i in range(8)}

    def later():
        time.sleep(0.4)
        with open(paths[3] + ".tmp", "w") as fh:
            fh.write(f"{1 << 30}\n")
        os.replace(paths[3] + ".tmp", paths[3])

    t = threading.Thread(target=later)
    t.start()
    got = hbm.settle(str(tmp_path), quiet_s=5.0, poll_s=0.005, timeout_s=10, floor=floor)
    t.join()
    assert got["reached_floor"] and got["waited_s"] >= 0.4 and got["floor"] == floor


def test_stop_phases_are_the_gpu_agents_max_then_mean_over_steps():
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("bench_mod2", os.path.join(os.path.dirname(__file__), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    results = [
        {"agent_stop_ms": {"mi355x-0": {"rccl_drain": 10.0, "total": 20.0}, "mi355x-1": {"rccl_drain": 30.0, "total": 40.0},
                           "control-plane": {"rccl_drain": 999.0, "total": 999.0}}},
        {"agent_stop_ms": {"mi355x-0": {"rccl_drain": 50.0, "total": 60.0}, "mi355x-1": None}},
        {},
    ]
    assert bench._stop_phases(results) == {"rccl_drain": 40.0, "total": 50.0}
    assert bench._stop_phases([{}]) == {}


class _Clock:
    def __init__(self):
        self.t = 0.0

    def __call__(self):
        return self.t


def _run(bench, budget, clock, warmup, steps, settle_s, step_s, warm_steps=2):
    """The bench's loop against a fake clock: each settle takes ``settle_s`` (capped by the
    budget, as ``hbm.settle(timeout_s=...)`` caps it), each step ``step_s``."""
    waited = []
    total = warmup + steps
    for k in range(total):
        w = settle_s if budget.settle_cap_s is None else min(settle_s, budget.settle_cap_s)
        waited.append(w)
        clock.t += w + step_s
        budget.record(w, step_s, settle_cut=w < settle_s)  # a capped wait ends at its limit
        budget.plan(total - k - 1, warm_steps + 1)
    if budget.warm_allowed:
        clock.t += (warm_steps + 1) * (settle_s + step_s)
    return waited


def test_run_budget_keeps_everything_when_it_fits():
    import bench

    clock = _Clock()
    b = bench.RunBudget(420, t0=0.0, clock=clock)
    waited = _run(bench, b, clock, 5, 20, settle_s=8.4, step_s=2.3)  # the 1-GPU box of round 5
    assert b.shed == [] and b.warm_allowed and b.settle_cap_s is None and waited == [8.4] * 25
    assert clock.t < 420


def test_run_budget_sheds_warm_creates_then_caps_slow_settles():
    """A node whose driver clears 8 cards one after another: ~67 s per settle.  The warm
    creates go first, then each settle is capped so the run ends inside the budget; the
    25 cold steps all run."""
    import bench

    clock = _Clock()
    b = bench.RunBudget(420, t0=0.0, clock=clock)
    waited = _run(bench, b, clock, 5, 20, settle_s=67.0, step_s=3.0)
    assert b.shed == ["warm_creates", "hbm_settle_capped"] and not b.warm_allowed
    assert len(waited) == 25 and waited[0] == 67.0 and max(waited[2:]) < 67.0
    assert clock.t + b.TAIL_S <= 420 + 1e-6
    rep = b.report()
    assert rep["budget_s"] == 420 and rep["shed"] == b.shed and rep["settle_cap_s"] == min(b.caps_used)


def test_run_budget_sheds_only_the_warm_creates_when_that_suffices():
    import bench

    clock = _Clock()
    b = bench.RunBudget(330, t0=0.0, clock=clock)
    waited = _run(bench, b, clock, 5, 20, settle_s=9.0, step_s=2.5, warm_steps=10)
    assert b.shed == ["warm_creates"] and b.settle_cap_s is None and waited == [9.0] * 25


def test_run_budget_zero_is_off():
    import bench

    clock = _Clock()
    b = bench.RunBudget(0, t0=0.0, clock=clock)
    _run(bench, b, clock, 5, 20, settle_s=100.0, step_s=3.0)
    assert b.shed == [] and b.warm_allowed and b.projected_s > 0


def test_bench_settle_passes_the_budget_cap_to_the_wait():
    import bench

    seen = []

    class FakeHBM:
        def settle(self, cards, floor, **kw):
            seen.append(kw)
            return {"waited_s": 0.0, "floor_by_card": {}, "reached_floor": True, "timed_out": False}

    bench.settle_cards(FakeHBM(), ["card0"], [None], resident=False)
    bench.settle_cards(FakeHBM(), ["card0"], [None], resident=False, timeout_s=3.5)
    assert seen == [{}, {"timeout_s": 3.5}]


def test_run_budget_decides_afresh_after_a_slow_cold_first_step():
    """A fresh box's first step can be slow (a cold code-object cache, a first import): the
    cap it causes is lifted once ordinary steps show the run fits, and the warm creates run
    when the time is there at the end."""
    import bench

    clock = _Clock()
    b = bench.RunBudget(480, t0=0.0, clock=clock)
    clock.t = 120.0  # a slow first import on a fresh box
    waited, total = [], 25
    for k in range(total):
        w = 8.4 if b.settle_cap_s is None else min(8.4, b.settle_cap_s)
        step = 60.0 if k == 0 else 2.3
        waited.append(w)
        clock.t += w + step
        b.record(w, step, settle_cut=w < 8.4)
        b.plan(total - k - 1, 3)
    assert b.caps_used and b.caps_used[0] < 8.4  # the cold first step made it cap ...
    assert waited[-1] == 8.4 and b.settle_cap_s is None  # ... and ordinary steps lifted the cap
    assert b.warm_allowed and b.shed == ["hbm_settle_capped"]
    assert b.report()["capped_settles"] == len(b.caps_used) < 5


@settings(max_examples=300, deadline=None)
@given(settle=st.floats(0.0, 120.0), step=st.floats(0.5, 10.0), n=st.integers(1, 30), warm=st.sampled_from([0, 3]),
       budget=st.floats(60.0, 600.0))
def test_run_budget_holds_whenever_the_steps_themselves_fit(settle, step, n, warm, budget):
    """A simulated run whose every settle wants ``settle`` seconds (the driver's clearing:
    up to the settle's own 120 s limit) and every step takes ``step``.  Whenever the work
    that cannot be shed fits -- the first settle (before any projection), every step and
    the tail -- the run ends inside the budget, whatever the settles want; and all ``n``
    steps run."""
    from hypothesis import assume

    import bench

    assume(settle + n * step + bench.RunBudget.TAIL_S <= budget)
    now = [0.0]
    b = bench.RunBudget(budget, t0=0.0, clock=lambda: now[0])
    ran = 0
    for i in range(n):
        waited = settle if b.settle_cap_s is None else min(settle, b.settle_cap_s)
        now[0] += waited + step
        ran += 1
        b.record(waited, step, settle_cut=waited < settle)
        b.plan(n - i - 1, warm)
    if warm and b.warm_allowed:
        for _ in range(warm):
            now[0] += (settle if b.settle_cap_s is None else min(settle, b.settle_cap_s)) + step
    now[0] += bench.RunBudget.TAIL_S
    assert ran == n
    assert now[0] <= budget + 1e-6, (now[0], b.report())
    assert b.settle_cap_s is None or b.settle_cap_s >= 0.0


@pytest.mark.parametrize("argv", [["--steps", "0"], ["--steps", "-2"], ["--gpus", "0"], ["--warmup", "-1"],
                                  ["--workers", "0"], ["--rccl-mib", "0"], ["--warm-steps", "-1"],
                                  ["--time-budget", "nan"], ["--time-budget", "-5"], ["--link-min-gbps", "inf"],
                                  ["--steps", "3.5"], ["--gpus", "eight"]])
def test_bench_refuses_counts_that_mean_nothing(argv, capsys):
    """`--steps 0` timed nothing and divided by zero; a negative warm-up or budget meant
    nothing.  argparse refuses them (exit 2) before anything starts."""
    import bench

    with pytest.raises(SystemExit) as exc:
        bench.parse_args(argv)
    assert exc.value.code == 2
    assert "argument --" in capsys.readouterr().err


def test_bench_accepts_the_drivers_command_lines():
    import bench

    for argv in ([], ["--gpus", "8", "--steps", "20", "--warmup", "5"], ["--steps", "1", "--warmup", "0"],
                 ["--time-budget", "0", "--warm-steps", "0", "--link-min-gbps", "38.5"]):
        args = bench.parse_args(argv)
        assert args.steps >= 1 and args.warmup >= 0 and args.gpus >= 1
