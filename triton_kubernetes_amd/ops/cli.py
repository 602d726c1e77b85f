"""Command line for the native probes (what a node bootstrap or an operator runs).

    python -m triton_kubernetes_amd.ops.cli burnin [--device N|--all] [--level quick|full]
    python -m triton_kubernetes_amd.ops.cli topology
    python -m triton_kubernetes_amd.ops.cli labels
    python -m triton_kubernetes_amd.ops.cli health [--max-uncorrectable N] [--max-bad-pages N|auto] [--source sysfs|amdsmi]
    python -m triton_kubernetes_amd.ops.cli metrics [--node NAME] [--max-uncorrectable N] [--max-bad-pages N|auto] [--source ...]
    python -m triton_kubernetes_amd.ops.cli rccl-local [--ngpus N]
    python -m triton_kubernetes_amd.ops.cli links [--min-frac F] [--min-gbps G] [--method kernel-read|sdma-copy] [--mib M]
    python -m triton_kubernetes_amd.ops.cli hbm|mfma [...] [--clock]
    python -m triton_kubernetes_amd.ops.cli rccl-slim [--source DIR] [--root DIR] [--no-verify]
    python -m triton_kubernetes_amd.ops.cli gemm [--size N] [--reps R] [--schedule staggered|single-barrier] [--dtype bf16|fp8]

Every command prints one JSON document (``metrics``: Prometheus text); the exit status is
non-zero when the GPU(s) fail the gate.
"""

import argparse
import json
import sys
from typing import Sequence


def main(argv: Sequence[str] = ()) -> int:
    """The command's exit code.  A refusal (a bad threshold, a GEMM size the kernel does not
    take, a native library that is not there, a probe that failed) is one ``tk-gpu: ...``
    line on stderr and exit 2, not a traceback."""
    from ..errors import TKError
    from .gemm import GemmError
    from .native import NativeUnavailable
    from .probe import ProbeError

    try:
        return _main(argv)
    except (TKError, GemmError, NativeUnavailable, ProbeError, ValueError) as exc:
        print(f"tk-gpu: {exc}", file=sys.stderr)
        return 2


def _num(lo, kind=int, above=False):
    """An argparse type: a finite ``kind`` >= ``lo`` (> ``lo`` with ``above``).  A negative
    size reached the native probes as a huge unsigned byte count."""
    import math

    def parse(text):
        try:
            v = kind(text)
        except ValueError:
            raise argparse.ArgumentTypeError(f"not a{'n integer' if kind is int else ' number'}: {text!r}")
        if not math.isfinite(v) or v < lo or (above and v == lo):
            raise argparse.ArgumentTypeError(f"must be {'>' if above else '>='} {lo}: {text!r}")
        return v

    parse.__name__ = kind.__name__
    return parse


def _collected(doc: dict) -> dict:
    """A topology document the collector finished; a node with no GPU to judge (status 2,
    as ``amdgpu-topo-labeller --health`` exits) is not a healthy one."""
    if doc.get("status", 0) != 0:
        from ..errors import TKError

        raise TKError(f"GPU collector failed (status {doc.get('status')}): {doc.get('error', 'no detail')}")
    return doc


def _main(argv: Sequence[str]) -> int:
    ap = argparse.ArgumentParser(prog="tk-gpu")
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("burnin")
    b.add_argument("--device", type=_num(0), default=0)
    b.add_argument("--all", action="store_true")
    b.add_argument("--level", default="full", choices=["quick", "full", "off"])
    sub.add_parser("topology")
    sub.add_parser("labels")
    hl = sub.add_parser("health", help="GPU RAS health: uncorrectable ECC errors, retired VRAM pages (node/health.py)")
    hl.add_argument("--max-uncorrectable", type=_num(0), default=0)
    hl.add_argument("--max-bad-pages", default="auto", help="a count, or auto (the driver's default threshold)")
    hl.add_argument("--source", default="sysfs", choices=["sysfs", "amdsmi"])
    mt = sub.add_parser("metrics", help="GPU health as Prometheus text (node/metrics.py; what the textfile timer writes)")
    mt.add_argument("--node", default="", help="the node label (default: the host name)")
    mt.add_argument("--max-uncorrectable", type=_num(0), default=0)
    mt.add_argument("--max-bad-pages", default="auto")
    mt.add_argument("--source", default="sysfs", choices=["sysfs", "amdsmi"])
    r = sub.add_parser("rccl-local")
    r.add_argument("--ngpus", type=_num(0), default=0)
    r.add_argument("--dtype", default="f32", choices=["f32", "bf16"])
    lk = sub.add_parser("links", help="per-link xGMI check: peer bandwidth of every ordered GPU pair")
    lk.add_argument("--min-frac", type=_num(0.0, float), default=0.5, help="fail below this fraction of the node median")
    lk.add_argument("--min-gbps", type=_num(0.0, float), default=None,
                    help="fail below this absolute GB/s (default: half of one link's ~76.8 GB/s one way)")
    lk.add_argument("--method", default="kernel-read", choices=["kernel-read", "sdma-copy"])
    lk.add_argument("--mib", type=_num(1), default=64, help="bytes per copy (MiB)")
    sl = sub.add_parser("rccl-slim", help="opt-in: prepare and verify the single-target (gfx950) RCCL copy")
    sl.add_argument("--source", default="")
    sl.add_argument("--no-verify", action="store_true", help="skip the GPU verification (the copy stays unused)")
    sl.add_argument("--root", default="")
    h = sub.add_parser("hbm")
    h.add_argument("--device", type=_num(0), default=0)
    h.add_argument("--gib", type=_num(0.0, float, above=True), default=4.0)
    h.add_argument("--blocks-per-cu", type=_num(1), default=16)
    m = sub.add_parser("mfma")
    m.add_argument("--device", type=_num(0), default=0)
    m.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "f32"])
    m.add_argument("--iters", type=_num(1), default=20000)
    m.add_argument("--blocks-per-cu", type=_num(1), default=2)
    g = sub.add_parser("gemm", help="checksum-verified GEMM screen (silent data corruption)")
    g.add_argument("--device", type=_num(0), default=0)
    g.add_argument("--size", type=_num(1), default=8192, help="M = N = K (a multiple of 256)")
    g.add_argument("--reps", type=_num(1), default=5)
    g.add_argument("--schedule", default="staggered", choices=["staggered", "single-barrier"],
                   help="GEMM main loop (single-barrier: the earlier loop, for A/B; bf16 only)")
    g.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                   help="operands: bf16, or fp8 e4m3 through the block-scaled MFMA")
    m.add_argument("--clock", action="store_true",
                   help="also report the in-kernel clock and FLOP/clk/SIMD (stamped diagnostic launch)")
    args = ap.parse_args(list(argv) or sys.argv[1:])

    if args.cmd == "burnin":
        from . import probe

        devs = range(probe.device_count()) if args.all else [args.device]
        results = [probe.run_burnin(d, args.level) for d in devs]
        print(json.dumps([r.to_json() for r in results], indent=2, default=str))
        return 0 if all(r.ok for r in results) else 1
    if args.cmd == "topology":
        from . import topo

        print(json.dumps(topo.discover(), indent=2))
        return 0
    if args.cmd == "labels":
        from ..node.labels import labels_from_topology
        from . import topo

        print(json.dumps(labels_from_topology(topo.discover()), indent=2, sort_keys=True))
        return 0
    if args.cmd == "health":
        from ..node.health import evaluate, limits_of
        from . import topo

        max_ue, max_bad = limits_of({"gpu_max_uncorrectable_ecc": args.max_uncorrectable,
                                     "gpu_max_retired_pages": args.max_bad_pages})
        doc = _collected(topo.native_topology("sysfs") if args.source == "sysfs" else topo.amdsmi_topology())
        verdict = evaluate(doc, max_ue, max_bad)
        print(json.dumps(verdict, indent=2))
        return 0 if verdict["status"] == "healthy" else 3
    if args.cmd == "metrics":
        import socket

        from ..node.health import evaluate, limits_of
        from ..node.metrics import gpu_metrics
        from . import topo

        max_ue, max_bad = limits_of({"gpu_max_uncorrectable_ecc": args.max_uncorrectable,
                                     "gpu_max_retired_pages": args.max_bad_pages})
        doc = _collected(topo.native_topology("sysfs") if args.source == "sysfs" else topo.amdsmi_topology())
        sys.stdout.write(gpu_metrics(evaluate(doc, max_ue, max_bad), args.node or socket.gethostname()))
        return 0
    if args.cmd == "rccl-local":
        from . import probe, rccl

        n = args.ngpus or probe.device_count()
        res = rccl.sweep_local(n, dtype=args.dtype)
        print(json.dumps(res.to_json(), indent=2))
        return 0 if res.ok else 1
    if args.cmd == "links":
        from ..node.labels import link_labels
        from . import probe

        n = probe.device_count()
        if n < 2:
            print(json.dumps({"skipped": "single GPU"}))
            return 0
        matrix = probe.link_matrix(range(n), args.mib << 20, method=args.method)
        verdict = link_labels(matrix, args.min_frac,
                              probe.DEFAULT_MIN_LINK_GBPS if args.min_gbps is None else args.min_gbps)
        print(json.dumps(dict(verdict, pairs=matrix["pairs"]), indent=2, sort_keys=True))
        return 1 if verdict["status"] == "degraded" else 0
    if args.cmd == "rccl-slim":
        from . import rccl_slim

        return rccl_slim.main((["--source", args.source] if args.source else [])
                              + (["--root", args.root] if args.root else []) + (["--no-verify"] if args.no_verify else []))
    if args.cmd == "hbm":
        from . import probe

        print(json.dumps(probe.hbm_bandwidth(args.device, int(args.gib * (1 << 30)), 5, args.blocks_per_cu)))
        return 0
    if args.cmd == "mfma":
        from . import probe

        res = probe.mfma_peak(args.device, args.dtype, args.iters, 3, args.blocks_per_cu)
        if args.clock:
            res["clock"] = probe.mfma_clock(args.device, args.dtype, args.iters, blocks_per_cu=args.blocks_per_cu)
        print(json.dumps(res))
        return 0
    if args.cmd == "gemm":
        from . import gemm

        gemm.set_schedule(args.schedule)
        res = gemm.screen(args.device, args.size, args.size, args.size, args.reps, dtype=args.dtype)
        print(json.dumps(dict(res.to_json(), schedule=args.schedule if args.dtype == "bf16" else "staggered")))
        return 0 if res.ok else 1
    return 2


if __name__ == "__main__":
    sys.exit(main())
