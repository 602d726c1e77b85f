#!/usr/bin/env python3
"""Fake ``ssh`` client: reachability, host keys and (optionally) remote execution.

A host is "up" when ``$FAKE_SSH_HOSTS/<host>/`` exists; that directory is its home and
``/etc/triton-kubernetes``.  Its host key is ``<dir>/host_key`` (``"<type> <base64>"``),
else one derived from its name.  A host that is down fails the way OpenSSH does: exit 255
with "connect to host ... No route to host".

A host may have several keys (``<dir>/host_keys``); it presents the one of the first
algorithm in the client's ``HostKeyAlgorithms`` (OpenSSH's default order, Ed25519 first,
without it), and ``UpdateHostKeys=yes`` pins the others after the first is verified.
Host keys are checked the way OpenSSH checks them, per key type, against
``-o UserKnownHostsFile=F`` with ``-o StrictHostKeyChecking=``:

* ``no``: not checked (nothing recorded);
* ``accept-new``: an unknown host's key is appended to F, a known host's must match;
* ``yes`` (or unset): it must be in F already.

A mismatch prints OpenSSH's "REMOTE HOST IDENTIFICATION HAS CHANGED" banner and
"Host key verification failed." and exits 255 before anything runs.  A ``ProxyCommand``
of the form ``ssh <opts> -W %h:%p user@bastion`` checks the bastion's key the same way
(with the hop's own options).

Commands: ``cat <file>`` prints the file from the host directory (``~/x`` and
``/etc/triton-kubernetes/x`` both map to ``<dir>/x``); with ``FAKE_SSH_EXEC=1`` the remote
command (or stdin for ``bash -s``) runs locally under ``bash`` -- with ``FAKE_SSH_HOST_ROOT=1``
with ``TK_HOST_ROOT=<dir>/root``, the host's filesystem for the scripts that honour it
(``node/cleanup.py``); otherwise anything else succeeds silently.  Every call is appended to ``$FAKE_SSH_LOG`` when set.
"""

import base64
import hashlib
import json
import os
import re
import shlex
import subprocess
import sys

WITH_VALUE = {"-o", "-i", "-J", "-p", "-l", "-F", "-E", "-b", "-c", "-m", "-L", "-R", "-D", "-W"}


def parse(argv):
    i, opts, flags = 0, {}, []
    while i < len(argv) and argv[i].startswith("-"):
        a = argv[i]
        if a in WITH_VALUE and i + 1 < len(argv):
            if a == "-o":
                k, _, v = argv[i + 1].partition("=")
                opts[k.lower()] = v
            else:
                flags.append((a, argv[i + 1]))
            i += 2
            continue
        flags.append((a, None))
        i += 1
    return opts, flags, argv[i:]


# OpenSSH's default host key algorithm order (Ed25519 first); rsa-sha2-* verify ssh-rsa keys
OPENSSH_DEFAULT_ALGS = ["ssh-ed25519", "ecdsa-sha2-nistp256", "ecdsa-sha2-nistp384", "ecdsa-sha2-nistp521",
                        "rsa-sha2-512", "rsa-sha2-256"]


def host_keys(host):
    """Every key of the host: ``<dir>/host_keys`` (one per line), ``<dir>/host_key``, or one
    ed25519 key derived from its name."""
    d = os.path.join(os.environ.get("FAKE_SSH_HOSTS", "/nonexistent"), host)
    for name in ("host_keys", "host_key"):
        path = os.path.join(d, name)
        if os.path.exists(path):
            return [" ".join(ln.split()[:2]) for ln in open(path, encoding="utf-8") if ln.strip()]
    blob = base64.b64encode(b"\x00\x00\x00\x0bssh-ed25519\x00\x00\x00\x20" + hashlib.sha256(host.encode()).digest())
    return ["ssh-ed25519 " + blob.decode()]


def host_key(host, opts=None):
    """The key the host presents: the first of the client's HostKeyAlgorithms (OpenSSH's
    default order without the option) the host has a key for."""
    keys = host_keys(host)
    algs = (opts or {}).get("hostkeyalgorithms")
    for alg in (algs.split(",") if algs else OPENSSH_DEFAULT_ALGS):
        ktype = "ssh-rsa" if alg.startswith("rsa-sha2-") else alg
        for k in keys:
            if k.split(" ", 1)[0] == ktype:
                return k
    return keys[0]


def check_key(host, opts):
    """None when the connection may proceed, else OpenSSH's error text.  As OpenSSH: a
    pinned key of the presented key's type must match; no pinned key of that type is a new
    key (accept-new adds it); UpdateHostKeys=yes then pins the host's other keys."""
    mode = opts.get("stricthostkeychecking", "yes").lower()
    if mode == "no":
        return None
    path = opts.get("userknownhostsfile", os.path.expanduser("~/.ssh/known_hosts")).split()[0]
    want = host_key(host, opts)
    pinned = []
    if path != "/dev/null" and os.path.exists(path):
        for line in open(path, encoding="utf-8"):
            parts = line.split()
            if len(parts) >= 3 and host in parts[0].split(",") and parts[1] == want.split(" ", 1)[0]:
                pinned.append(f"{parts[1]} {parts[2]}")
    if pinned:
        if want in pinned:
            _update_host_keys(host, opts, path)
            return None
        return ("@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@\n"
                "@    WARNING: REMOTE HOST IDENTIFICATION HAS CHANGED!     @\n"
                "@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@@\n"
                f"Host key for {host} has changed and you have requested strict checking.\n"
                "Host key verification failed.\n")
    if mode in ("accept-new", "off") and path != "/dev/null":
        with open(path, "a", encoding="utf-8") as fh:
            fh.write(f"{host} {want}\n")
        _update_host_keys(host, opts, path)
        return None
    return f"No ED25519 host key is known for {host} and you have requested strict checking.\n" \
           "Host key verification failed.\n"


def _update_host_keys(host, opts, path):
    if opts.get("updatehostkeys", "no").lower() != "yes" or path == "/dev/null":
        return
    have = set()
    if os.path.exists(path):
        have = {" ".join(ln.split()[:3]) for ln in open(path, encoding="utf-8") if ln.strip()}
    with open(path, "a", encoding="utf-8") as fh:
        for k in host_keys(host):
            if f"{host} {k}" not in have:
                fh.write(f"{host} {k}\n")


def main() -> int:
    opts, flags, rest = parse(sys.argv[1:])
    if not rest:
        sys.stderr.write("usage: ssh destination [command]\n")
        return 255
    dest, command = rest[0], " ".join(rest[1:])
    host = dest.rsplit("@", 1)[-1]
    log = os.environ.get("FAKE_SSH_LOG")
    if log:
        with open(log, "a", encoding="utf-8") as fh:
            fh.write(json.dumps({"opts": opts, "flags": flags, "host": host, "command": command}) + "\n")
    hosts = os.environ.get("FAKE_SSH_HOSTS", "/nonexistent")
    proxy = opts.get("proxycommand")
    if proxy:  # the hop: its own options, its own key check
        p_opts, _, p_rest = parse(shlex.split(proxy)[1:])
        bastion = p_rest[0].rsplit("@", 1)[-1] if p_rest else ""
        if not os.path.isdir(os.path.join(hosts, bastion)):
            sys.stderr.write(f"ssh: connect to host {bastion} port 22: No route to host\n")
            return 255
        err = check_key(bastion, p_opts)
        if err:
            sys.stderr.write(err)
            return 255
    home = os.path.join(hosts, host)
    if not os.path.isdir(home):
        sys.stderr.write(f"ssh: connect to host {host} port 22: No route to host\n")
        return 255
    err = check_key(host, opts)
    if err:
        sys.stderr.write(err)
        return 255
    if os.environ.get("FAKE_SSH_EXEC") == "1" and command:
        env = None
        if os.environ.get("FAKE_SSH_HOST_ROOT") == "1":  # the host's filesystem: <dir>/root
            env = dict(os.environ, TK_HOST_ROOT=os.path.join(home, "root"))
            os.makedirs(env["TK_HOST_ROOT"], exist_ok=True)
        if command.strip() == "bash -s":
            return subprocess.run(["bash", "-s"], stdin=sys.stdin, env=env).returncode
        return subprocess.run(["bash", "-c", command], env=env).returncode
    for m in re.finditer(r"\bcat\s+(\S+)", command):
        path = os.path.join(home, os.path.basename(m.group(1)))
        if os.path.exists(path):
            sys.stdout.write(open(path, encoding="utf-8").read())
        elif "2>/dev/null" not in command[m.end():m.end() + 12]:
            sys.stderr.write(f"cat: {m.group(1)}: No such file or directory\n")
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
