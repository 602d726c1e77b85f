#!/usr/bin/env python3
"""Fake ``terraform`` executable (the Terraform double SURVEY.md §4 calls for).

Behaviour by sub-command:

* ``version``            prints ``Terraform v$FAKE_TF_VERSION`` (default 1.5.7)
* ``init``               records, succeeds
* ``apply``              records; writes a tfstate with fake values for every
                         root ``output`` of ``main.tf.json`` to the local backend path
* ``destroy``            records, succeeds
* ``output``             ``-json`` (root outputs) or ``-module=<key>`` (0.11 style)

Every call appends ``{"argv": [...], "cwd": ..., "doc": <main.tf.json>}`` to
``$FAKE_TF_LOG``.  ``FAKE_TF_FAIL=<subcommand>`` makes that sub-command exit 1.
"""

import json
import os
import sys


def main() -> int:
    argv = sys.argv[1:]
    cmd = argv[0] if argv else ""
    doc = {}
    if os.path.exists("main.tf.json"):
        with open("main.tf.json", "r", encoding="utf-8") as fh:
            doc = json.load(fh)
    log = os.environ.get("FAKE_TF_LOG")
    if log:
        with open(log, "a", encoding="utf-8") as fh:
            fh.write(json.dumps({"argv": argv, "cwd": os.getcwd(), "doc": doc}) + "\n")
    if os.environ.get("FAKE_TF_FAIL") == cmd:
        sys.stderr.write(f"Error: fake failure of {cmd}\n")
        return 1
    version = os.environ.get("FAKE_TF_VERSION", "1.5.7")
    backend_path = (((doc.get("terraform") or {}).get("backend") or {}).get("local") or {}).get("path")
    if cmd == "version":
        print(f"Terraform v{version}\non linux_amd64")
        return 0
    if cmd == "apply":
        outputs = {}
        for name, spec in (doc.get("output") or {}).items():
            outputs[name] = {"value": f"fake-{name}", "type": "string"}
        if backend_path:
            os.makedirs(os.path.dirname(backend_path), exist_ok=True)
            with open(backend_path, "w", encoding="utf-8") as fh:
                json.dump({"version": 4, "outputs": outputs}, fh)
        print("Apply complete!")
        return 0
    if cmd == "output":
        state = {}
        if backend_path and os.path.exists(backend_path):
            with open(backend_path, "r", encoding="utf-8") as fh:
                state = json.load(fh)
        outs = state.get("outputs", {})
        module = next((a.split("=", 1)[1] for a in argv if a.startswith("-module=")), None)
        if module is None and "-module" in argv:
            module = argv[argv.index("-module") + 1]
        if module:
            outs = {k[len(module) + 2:]: v for k, v in outs.items() if k.startswith(module + "__")}
        if "-json" in argv:
            print(json.dumps(outs))
        else:
            for k in sorted(outs):
                print(f"{k} = {outs[k]['value']}")
        return 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
