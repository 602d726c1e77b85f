#!/usr/bin/env python3
"""Fake ``docker`` CLI with Docker's own filter semantics and a container table per host.

The RKE1 teardown (``node/cleanup.py``) decides what to remove from what ``docker ps``
tells it, so the double must answer as Docker does -- the round-5 stub answered "yes" to
any filter and hid that ``--filter ancestor=rancher/rancher-agent`` (untagged: Docker
resolves it to ``rancher/rancher-agent:latest``) matches no agent that runs a tagged image.
Nothing here imports ``triton_kubernetes_amd``.

State: ``$TK_HOST_ROOT/var/lib/docker/fake-containers.json`` (a list of
``{"id", "name", "image", "labels", "args"}``).  Without a host root it keeps no state and
every command succeeds with empty output: it never touches the machine it runs on.

* ``ps [-a] [-q] [--filter F]... [--format T]``: ``label=K`` / ``label=K=V`` (the container
  has the label), ``ancestor=IMG`` (the container's image, both sides normalised: an
  untagged reference means ``:latest``, ``docker.io/`` and ``library/`` are implied),
  ``name=N`` (substring of the name).  Several filters of one kind are OR-ed, of different
  kinds AND-ed.  ``--format`` expands ``{{.ID}}``, ``{{.Image}}``, ``{{.Names}}`` and
  ``{{.Labels}}`` (``k=v,k=v``).
* ``rm -f ID|NAME...``: removes them ("No such container" for an unknown one, exit 1).
* ``run -d [--name N] [--label K=V]... [opts] IMAGE [args]``: adds a container (a name
  already in use: Docker's "Conflict", exit 125).  An image of repository
  ``rancher/rancher-agent`` (any registry, any tag) models the RKE1 join: the agent
  container, then what Rancher has RKE start for the node -- ``kubelet`` and
  ``kube-proxy`` (label ``io.rancher.rke.container.name``) and the kubelet's pod
  containers (``k8s_*``, label ``io.kubernetes.pod.namespace``, each pod with its
  ``k8s_POD_*`` sandbox).  RKE's fixed container names make a second cluster's join on a
  host that still has the first cluster's containers fail as Docker fails it; an agent of
  another server or token still running refuses the join too (it would keep the node
  registered with its old cluster).
* anything else (``login``, ``info``, ...): exit 0.
"""

import json
import os
import secrets
import sys

AGENT_REPO = "rancher/rancher-agent"
RKE_LABEL = "io.rancher.rke.container.name"
POD_NS_LABEL = "io.kubernetes.pod.namespace"
POD_NAME_LABEL = "io.kubernetes.pod.name"


def _state_path():
    root = os.environ.get("TK_HOST_ROOT", "")
    if not root or root == "/":
        return None
    return os.path.join(root, "var/lib/docker/fake-containers.json")


def load():
    p = _state_path()
    if p is None or not os.path.exists(p):
        return []
    with open(p, "r", encoding="utf-8") as fh:
        return json.load(fh)


def save(table):
    p = _state_path()
    if p is None:
        return
    os.makedirs(os.path.dirname(p), exist_ok=True)
    with open(p + ".tmp", "w", encoding="utf-8") as fh:
        json.dump(table, fh, indent=1)
    os.replace(p + ".tmp", p)


def normalise(ref):
    """Docker's reference normalisation: ``(repository, tag)``; ``docker.io/`` and
    ``library/`` implied, no tag means ``latest`` (a digest is kept as the tag)."""
    ref, digest = (ref.split("@", 1) + [""])[:2]
    last = ref.rsplit("/", 1)[-1]
    tag = ""
    if ":" in last:
        ref, tag = ref.rsplit(":", 1)
    first = ref.split("/", 1)[0]
    if "/" not in ref or not ("." in first or ":" in first or first == "localhost"):
        ref = "docker.io/" + ref
    if ref.count("/") == 1:
        ref = ref.replace("docker.io/", "docker.io/library/", 1)
    return ref, ("@" + digest) if digest else (tag or "latest")


def repository(ref):
    return normalise(ref)[0]


def is_agent(ref):
    """An image of the agent's repository, from any registry."""
    return repository(ref).endswith("/" + AGENT_REPO)


def _match(c, filters):
    kinds = {}
    for f in filters:
        k, _, v = f.partition("=")
        kinds.setdefault(k, []).append(v)
    for kind, values in kinds.items():
        ok = False
        for v in values:
            if kind == "label":
                key, eq, val = v.partition("=")
                ok = ok or (key in c["labels"] and (not eq or c["labels"][key] == val))
            elif kind == "ancestor":
                ok = ok or normalise(c["image"]) == normalise(v)
            elif kind == "name":
                ok = ok or v in c["name"]
            else:
                sys.stderr.write(f'Error response from daemon: invalid filter \'{kind}\'\n')
                sys.exit(1)
        if not ok:
            return False
    return True


def _format(c, tmpl):
    labels = ",".join(f"{k}={v}" for k, v in sorted(c["labels"].items()))
    return (tmpl.replace("{{.ID}}", c["id"]).replace("{{.Image}}", c["image"]).replace("{{.Names}}", c["name"])
            .replace("{{.Labels}}", labels))


def ps(argv):
    filters, fmt, quiet, i = [], None, False, 0
    while i < len(argv):
        a = argv[i]
        if a in ("-a", "--all"):
            pass
        elif a in ("-q", "--quiet"):
            quiet = True
        elif a in ("-aq", "-qa"):
            quiet = True
        elif a in ("--filter", "-f"):
            i += 1
            filters.append(argv[i])
        elif a.startswith("--filter="):
            filters.append(a.split("=", 1)[1])
        elif a == "--format":
            i += 1
            fmt = argv[i]
        elif a.startswith("--format="):
            fmt = a.split("=", 1)[1]
        i += 1
    for c in load():
        if _match(c, filters):
            print(c["id"] if quiet else _format(c, fmt or "{{.ID}} {{.Image}} {{.Names}}"))
    return 0


def rm(argv):
    targets = [a for a in argv if not a.startswith("-")]
    table = load()
    rc = 0
    for t in targets:
        hit = [c for c in table if c["id"] == t or c["name"] == t or c["id"].startswith(t)]
        if not hit:
            sys.stderr.write(f"Error response from daemon: No such container: {t}\n")
            rc = 1
            continue
        table = [c for c in table if c not in hit]
        print(t)
    save(table)
    return rc


def _add(table, image, name, labels, args):
    if any(c["name"] == name for c in table):
        sys.stderr.write(f'docker: Error response from daemon: Conflict. The container name "/{name}" is already in '
                         f"use by container. You have to remove (or rename) that container to be able to reuse "
                         f"that name.\n")
        sys.exit(125)
    cid = secrets.token_hex(6)
    table.append({"id": cid, "name": name, "image": image, "labels": labels, "args": args})
    return cid


def run(argv):
    name, labels, i = "", {}, 0
    opts_with_value = {"-v", "--volume", "-e", "--env", "--net", "--network", "--restart", "-p", "--env-file"}
    while i < len(argv) and argv[i].startswith("-"):
        a = argv[i]
        if a == "--name":
            i += 1
            name = argv[i]
        elif a.startswith("--name="):
            name = a.split("=", 1)[1]
        elif a in ("--label", "-l"):
            i += 1
            k, _, v = argv[i].partition("=")
            labels[k] = v
        elif a in opts_with_value:
            i += 1
        i += 1
    if i >= len(argv):
        sys.stderr.write('"docker run" requires at least 1 argument.\n')
        return 1
    image, args = argv[i], argv[i + 1:]
    table = load()
    if is_agent(image):
        server = args[args.index("--server") + 1] if "--server" in args else ""
        token = args[args.index("--token") + 1] if "--token" in args else ""
        for c in table:
            if is_agent(c["image"]) and not c["name"].startswith("k8s_"):
                a = c["args"]
                other = (a[a.index("--server") + 1] if "--server" in a else "",
                         a[a.index("--token") + 1] if "--token" in a else "")
                if other != (server, token):
                    sys.stderr.write(f"rancher-agent: another rancher-agent ({c['image']}, container {c['id']}) is "
                                     f"still running on this host, registered with {other[0]}: the node would stay "
                                     f"in its old cluster\n")
                    return 1
        cid = _add(table, image, name or f"agent_{secrets.token_hex(3)}", labels, args)
        # what RKE then runs for the node: fixed-name system containers and the kubelet's pods
        hyperkube = "rancher/hyperkube:v1.28.15-rancher1"
        for svc in ("kubelet", "kube-proxy"):
            _add(table, hyperkube, svc, {RKE_LABEL: svc}, [])
        for pod, img in (("kube-flannel-x1", "rancher/mirrored-flannel-flannel:v0.25.1"),
                         ("cattle-node-agent-x2", image)):
            ns = "kube-system" if "flannel" in pod else "cattle-system"
            pl = {POD_NS_LABEL: ns, POD_NAME_LABEL: pod}
            _add(table, "rancher/mirrored-pause:3.7", f"k8s_POD_{pod}_{ns}_0", dict(pl), [])
            _add(table, img, f"k8s_{pod.rsplit('-', 1)[0]}_{pod}_{ns}_0", dict(pl), [])
        save(table)
        print(cid)
        return 0
    cid = _add(table, image, name or f"c_{secrets.token_hex(3)}", labels, args)
    save(table)
    print(cid)
    return 0


def main():
    argv = sys.argv[1:]
    while argv and argv[0].startswith("-"):  # global options (-H, --config ...)
        argv = argv[2:] if argv[0] in ("-H", "--host", "--config") else argv[1:]
    cmd, rest = (argv[0], argv[1:]) if argv else ("", [])
    if cmd == "ps":
        return ps(rest)
    if cmd == "rm":
        return rm(rest)
    if cmd == "run":
        return run(rest)
    if cmd == "container" and rest[:1] == ["ls"]:
        return ps(rest[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
