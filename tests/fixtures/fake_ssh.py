#!/usr/bin/env python3
"""Fake ``ssh`` client for the programs Terraform's ``data "external"`` sources run.

A host is "up" when ``$FAKE_SSH_HOSTS/<host>/`` exists; that directory is its home and
``/etc/triton-kubernetes``.  ``cat <file>`` commands print the file from there (``~/x``
and ``/etc/triton-kubernetes/x`` both map to ``<dir>/x``); any other command succeeds
silently.  A host that is down fails the way OpenSSH does: exit 255 with "connect to host
... No route to host".  Options (``-o``, ``-i``, ``-J`` …) are accepted and ignored, but
every call is appended to ``$FAKE_SSH_LOG`` when set.
"""

import json
import os
import re
import sys

WITH_VALUE = {"-o", "-i", "-J", "-p", "-l", "-F", "-E", "-b", "-c", "-m", "-L", "-R", "-D", "-W"}


def main() -> int:
    argv = sys.argv[1:]
    i, opts = 0, []
    while i < len(argv) and argv[i].startswith("-"):
        opts.append(argv[i])
        if argv[i] in WITH_VALUE and i + 1 < len(argv):
            opts.append(argv[i + 1])
            i += 1
        i += 1
    if i >= len(argv):
        sys.stderr.write("usage: ssh destination [command]\n")
        return 255
    dest, command = argv[i], " ".join(argv[i + 1:])
    host = dest.rsplit("@", 1)[-1]
    log = os.environ.get("FAKE_SSH_LOG")
    if log:
        with open(log, "a", encoding="utf-8") as fh:
            fh.write(json.dumps({"opts": opts, "host": host, "command": command}) + "\n")
    home = os.path.join(os.environ.get("FAKE_SSH_HOSTS", "/nonexistent"), host)
    if not os.path.isdir(home):
        sys.stderr.write(f"ssh: connect to host {host} port 22: No route to host\n")
        return 255
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
