"""HBM release backlog: wait until the kernel driver has finished clearing freed VRAM.

The amdgpu driver clears VRAM that a process releases before it hands that memory out
again (~35 GB/s per GPU, ``profiles/round4/alloc_probe.jsonl``).  Until the clear is done
the memory is still accounted as used in the driver's VRAM manager
(``/sys/class/drm/card*/device/mem_info_vram_used``), and an allocation that needs it
waits: right after a full burn-in released ~300 GB, the next 16 GiB ``hipMalloc`` waited
~6 s for the whole backlog.

A node entering service starts with its HBM clear.  The bench therefore waits, between
timed steps and outside the timed region, until the previous step's release has settled
(:func:`settle`), so that a step is never charged for the clearing of its predecessor's
memory.  Pure sysfs: no HIP call, so the waiting process does not touch the GPU.
"""

import glob
import os
import time
from typing import Any, Dict, Iterable, List, Optional, Tuple, Union

DRM_ROOT = "/sys/class/drm"


def cards_for_pci(addresses: Iterable[Tuple[int, int, int]], drm_root: str = DRM_ROOT) -> List[str]:
    """The DRM cards (``cardN``) of the GPUs at PCI ``(domain, bus, device)``: the GPUs this
    process can see.  A shared host lists every GPU under ``/sys/class/drm``, other
    tenants' too, whose allocations and releases must not be mistaken for ours."""
    want = {(int(d), int(b), int(v)) for d, b, v in addresses}
    out: List[str] = []
    for dev in sorted(glob.glob(os.path.join(drm_root, "card*", "device"))):
        card = dev.split(os.sep)[-2]
        if "-" in card:
            continue
        bdf = os.path.basename(os.path.realpath(dev))  # e.g. 0000:75:00.0
        try:
            dom, bus, rest = bdf.split(":")
            key = (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16))
        except ValueError:
            continue
        if key in want:
            out.append(card)
    return out


def vram_used(drm_root: str = DRM_ROOT, cards: Optional[Iterable[str]] = None) -> Dict[str, int]:
    """``mem_info_vram_used`` of the amdgpu cards under ``drm_root`` (bytes, by card): every
    card, or the ``cards`` named."""
    only = set(cards) if cards is not None else None
    out: Dict[str, int] = {}
    for path in sorted(glob.glob(os.path.join(drm_root, "card*", "device", "mem_info_vram_used"))):
        card = path.split(os.sep)[-3]
        if "-" in card:  # connectors (card0-DP-1) share the device directory
            continue
        if only is not None and card not in only:
            continue
        try:
            with open(path, "r", encoding="ascii") as fh:
                out[card] = int(fh.read().strip() or 0)
        except (OSError, ValueError):
            continue
    return out


def settle(drm_root: str = DRM_ROOT, quiet_s: float = 5.0, poll_s: float = 0.02, timeout_s: float = 120.0,
           floor: Optional[Union[int, Dict[str, int]]] = None, slack: Optional[int] = None,
           cards: Optional[Iterable[str]] = None) -> Dict[str, Any]:
    """Block until the used VRAM of ``cards`` (default: every card) is back at ``floor`` --
    the clean level an earlier call measured -- or, without a floor or when it is not
    reached, until none of their ``mem_info_vram_used`` dropped for ``quiet_s`` seconds.
    ``floor`` per card (a dict, ``floor_by_card`` of an earlier call): every card within
    ``slack`` (default 1 GiB) of its own level, so one card still clearing a large release
    is waited for whatever the others do.  ``floor`` as one number: the sum over the cards
    within ``slack`` (default 1 GiB per card).  Returns what it waited for, ``floor`` (the
    lowest level seen, in the form given) and ``floor_by_card``.  No cards: returns at once.

    The floor is what makes the wait reliable: a process that exits leaves its memory to
    the driver, which returns it (cleared) only later, a whole allocation at a time -- a
    16 GiB one ~0.5 s after the previous (``profiles/round5/vram_release.jsonl``) -- and the
    release may not have begun when the wait starts, so no quiet window alone can tell
    "nothing pending" from "not started yet"."""
    cards = list(cards) if cards is not None else None
    t0 = time.monotonic()
    first = vram_used(drm_root, cards)
    if not first:
        return {"waited_s": 0.0, "released_gib": 0.0, "cards": 0, "timed_out": False, "floor": 0,
                "floor_by_card": {}}
    last = dict(first)
    per_card = isinstance(floor, dict)
    if slack is None:
        slack = (1 << 30) if per_card else len(first) << 30
    low = dict(first)
    quiet_since = t0
    timed_out = False
    reached = False
    while True:
        for c, v in last.items():
            low[c] = min(low.get(c, v), v)
        if per_card:
            if all(v <= floor.get(c, v) + slack for c, v in last.items()):
                reached = True
                break
        elif floor is not None and sum(last.values()) <= floor + slack:
            reached = True
            break
        now = time.monotonic()
        if now - quiet_since >= quiet_s:
            break
        if now - t0 >= timeout_s:
            timed_out = True
            break
        time.sleep(poll_s)
        cur = vram_used(drm_root, cards)
        if any(cur.get(c, 0) < last.get(c, 0) for c in cur):
            quiet_since = time.monotonic()
        last = cur
    by_card = {c: min(v, floor[c]) if per_card and c in floor else v for c, v in low.items()}
    if per_card:
        out_floor: Union[int, Dict[str, int]] = by_card
    else:
        out_floor = min(sum(low.values()), floor) if floor is not None else sum(low.values())
    return {"waited_s": round(time.monotonic() - t0, 4),
            "released_gib": round(max(0, sum(first.values()) - sum(last.values())) / 2 ** 30, 2),
            "cards": len(first), "timed_out": timed_out, "reached_floor": reached,
            "floor": out_floor, "floor_by_card": by_card}
