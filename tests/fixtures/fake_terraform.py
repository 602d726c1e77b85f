#!/usr/bin/env python3
"""Fake ``terraform`` executable (the Terraform double SURVEY.md §4 calls for).

It models the parts of Terraform the CLI depends on — and the failures a real Terraform
of version ``$FAKE_TF_VERSION`` (default 1.5.7) reports — independently of the CLI's own
code (nothing here imports ``triton_kubernetes_amd``):

* ``version``  prints ``Terraform v$FAKE_TF_VERSION``;
* ``init``     rejects a backend type this version lacks (>= 1.3: ``manta``, ``etcd``,
               ``etcdv3``, ``artifactory``, ``swift`` — "Unsupported backend type"), a
               local module directory that does not exist, and a module whose
               ``required_version`` this version fails ("Unsupported Terraform Core
               version");
* ``apply`` / ``destroy`` / ``output`` validate the configuration first: from 0.15 a
               root output whose value is a module output the module declares
               ``sensitive = true`` must be ``sensitive`` itself ("Output refers to
               sensitive values");
* ``apply``    reads the prior state from the backend (``local`` path, relative to the
               work dir or absolute), adds one resource per module block, writes fake
               values for every root output, bumps ``serial`` and keeps ``lineage``;
* ``destroy``  removes the ``-target``-ed modules' resources (all without targets) and
               the outputs that read them;
* ``output``   ``-json`` (root outputs, with ``sensitive``) or ``-module=<key>`` (0.11);
* ``-var=name=value`` must name a declared root ``variable`` ("Value for undeclared
               variable");
* with ``FAKE_TF_EXTERNAL=1``, ``data "external"`` programs run during refresh —
               apply, plan, and destroy unless ``-refresh=false`` (targets + their
               dependencies) — and a failing program fails the command; module outputs
               that read a data source get its result.

* with ``FAKE_TF_HOSTS=<dir>``, bare-metal host modules (``var.host`` + a cluster
               registration token) model the host ``<dir>/<host>/root``: an apply records the
               join (what ``system-agent-install.sh`` leaves: ``/var/lib/rancher/agent/
               rancher2_connection_info.json``) and fails the module -- as the real join
               fails -- on a host still joined to another cluster; a destroy runs the
               module's destroy-time ``remote-exec`` (``when = destroy``) locally against
               that root (``TK_HOST_ROOT``) -- ``inline`` joined into one script, ``self.input``
               the values of the last apply -- honouring ``count = var.X ? 1 : 0`` and
               ``on_failure = continue``; a re-apply that takes such a ``count`` from 1 to 0
               destroys that instance, running its destroy-time provisioner, as Terraform does.

Every call appends ``{"argv", "cwd", "doc", "prior"}`` to ``$FAKE_TF_LOG`` (``prior``:
serial/lineage/modules of the state the command started from).  ``FAKE_TF_FAIL=<cmd>``
makes that sub-command fail *after* applying half of the new modules (apply) — a
partial state is written, as Terraform does.
"""

import json
import os
import re
import subprocess
import sys
import uuid

REMOVED_BACKENDS_1_3 = {"artifactory", "etcd", "etcdv3", "manta", "swift"}
# go-getter's forced getters (``<scheme>::<address>``) that Terraform's module installer has
GETTER_SCHEMES = {"git", "hg", "s3", "gcs", "http", "https", "file"}


def vtuple(text):
    parts = [int(x) for x in re.findall(r"\d+", text)[:3]]
    return tuple(parts + [0] * (3 - len(parts)))


def satisfied(version, constraint):
    for term in constraint.split(","):
        term = term.strip()
        if not term:
            continue
        m = re.match(r"^(=|!=|>=|<=|>|<|~>)?\s*v?([\d.]+)$", term)
        if not m:
            return False
        op, want = m.group(1) or "=", vtuple(m.group(2))
        ndots = m.group(2).count(".")
        ok = {"=": version == want, "!=": version != want, ">": version > want, ">=": version >= want,
              "<": version < want, "<=": version <= want}.get(op)
        if op == "~>":
            upper = (want[0] + 1, 0, 0) if ndots <= 1 else (want[0], want[1] + 1, 0)
            ok = want <= version < upper
        if not ok:
            return False
    return True


def fail(msg):
    sys.stderr.write(f"\nError: {msg}\n\n")
    return 1


def local_dir(source):
    path = source.split("?", 1)[0]
    return path if path.startswith(("/", "./", "../")) else None


def module_outputs(mod_dir):
    """{output: sensitive} declared in the module's .tf files (top-level output blocks)."""
    outs = {}
    for fn in sorted(os.listdir(mod_dir)):
        if not fn.endswith(".tf"):
            continue
        text = open(os.path.join(mod_dir, fn), encoding="utf-8").read()
        for m in re.finditer(r'^output\s+"([^"]+)"\s*\{(.*?)^\}', text, re.S | re.M):
            outs[m.group(1)] = re.search(r"^\s*sensitive\s*=\s*true\s*$", m.group(2), re.M) is not None
    return outs


def required_versions(mod_dir):
    out = []
    for fn in sorted(os.listdir(mod_dir)):
        if fn.endswith(".tf"):
            out += re.findall(r'required_version\s*=\s*"([^"]*)"', open(os.path.join(mod_dir, fn)).read())
    return out


def validate(doc, version):
    """Configuration errors Terraform reports before doing anything (plan/apply/output)."""
    modules = doc.get("module") or {}
    for key, mod in modules.items():
        d = local_dir(str(mod.get("source", "")))
        if d is not None and not os.path.isdir(d):
            return f"Unreadable module directory\n\nUnable to evaluate directory symlink: lstat {d}: no such file"
    if version >= (0, 15, 0):
        for name, out in (doc.get("output") or {}).items():
            m = re.fullmatch(r"\$\{module\.([^.}]+)\.([^.}]+)\}", str(out.get("value", "")))
            if not m or m.group(1) not in modules:
                continue
            d = local_dir(str(modules[m.group(1)].get("source", "")))
            if d is None:
                continue
            if module_outputs(d).get(m.group(2)) and out.get("sensitive") is not True:
                return ("Output refers to sensitive values\n\n  on main.tf.json line 1:\n"
                        f'  output "{name}"\n\nTo reduce the risk of accidentally exporting sensitive data that '
                        "was intended to be only internal, Terraform requires that any root module output "
                        "containing sensitive data be explicitly marked as sensitive, to confirm your intent.")
    return None


def state_path(doc):
    backend = ((doc.get("terraform") or {}).get("backend") or {})
    if "local" in backend:
        return backend["local"].get("path") or "terraform.tfstate"
    if backend:  # a remote backend this fake stands in for: keep it beside the log
        kind = next(iter(backend))
        base = os.environ.get("FAKE_TF_REMOTE") or os.path.join(os.getcwd(), ".remote")
        # a remote state is addressed by where it lives, not by whose credentials read it
        where = {k: v for k, v in backend[kind].items() if not re.search(r"key|secret|password|token", k)}
        ident = json.dumps(where, sort_keys=True)
        return os.path.join(base, kind, re.sub(r"[^A-Za-z0-9]+", "_", ident)[:120] + ".tfstate")
    return "terraform.tfstate"


def load_state(path):
    if os.path.exists(path):
        with open(path, "r", encoding="utf-8") as fh:
            return json.load(fh)
    return {}


def save_state(path, st):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w", encoding="utf-8") as fh:
        json.dump(st, fh)


def state_modules(st):
    return sorted({r["module"][len("module."):] for r in st.get("resources", []) if r.get("module")})


# --- data "external" (FAKE_TF_EXTERNAL=1) -------------------------------------------------------
#
# Terraform reads data sources while refreshing: every apply and plan, and every destroy
# unless -refresh=false (for a targeted destroy: the targets and what they depend on).  A
# data "external" source runs its program on the operator machine with the query as JSON
# on stdin; a non-zero exit fails the whole command.  Opt-in, because the programs of the
# packaged modules really reach out (ssh to the manager, HTTP to Rancher): a test turns it
# on with fakes for those on PATH / in process.  The query is evaluated by a tiny
# evaluator that knows var.X, local.X (one level) and string literals: enough for the
# modules' `query = { k = var.x }` / `query = local.request` (a merge of such maps).

def _braced(text, start):
    """The text between the brace at ``start`` and its match."""
    depth = 0
    for i in range(start, len(text)):
        if text[i] == "{":
            depth += 1
        elif text[i] == "}":
            depth -= 1
            if depth == 0:
                return text[start + 1:i]
    return text[start + 1:]


def _module_text(mod_dir):
    return "\n".join(open(os.path.join(mod_dir, fn), encoding="utf-8").read()
                     for fn in sorted(os.listdir(mod_dir)) if fn.endswith(".tf"))


def _locals(text):
    out = {}
    for m in re.finditer(r"^locals\s*\{", text, re.M):
        body = _braced(text, m.end() - 1)
        for a in re.finditer(r"^  (\w+)\s*=\s*", body, re.M):
            rest = body[a.end():]
            if rest[:1] in "({[" or rest.startswith("merge("):
                # a multi-line expression: up to the next top-level assignment
                nxt = re.search(r"^  \w+\s*=", rest, re.M)
                out[a.group(1)] = rest[:nxt.start()] if nxt else rest
            else:
                out[a.group(1)] = rest.split("\n", 1)[0].strip()
    return out


def _var_defaults(text):
    out = {}
    for m in re.finditer(r'^variable\s+"(\w+)"\s*\{', text, re.M):
        body = _braced(text, m.end() - 1)
        d = re.search(r'^\s*default\s*=\s*"((?:[^"\\]|\\.)*)"', body, re.M)
        if d:
            out[m.group(1)] = d.group(1)
            continue
        d = re.search(r'^\s*default\s*=\s*(true|false|-?\d+)\s*$', body, re.M)
        if d:  # a bool or number default, in its string form
            out[m.group(1)] = d.group(1)
    return out


def _value(expr, inputs, defaults, local_exprs, depth=0):
    expr = expr.strip()
    m = re.fullmatch(r"var\.(\w+)", expr)
    if m:
        v = inputs.get(m.group(1), defaults.get(m.group(1), ""))
        return v if isinstance(v, str) else json.dumps(v)
    m = re.fullmatch(r"local\.(\w+)", expr)
    if m and depth < 3 and m.group(1) in local_exprs:
        return _value(local_exprs[m.group(1)], inputs, defaults, local_exprs, depth + 1)
    m = re.fullmatch(r'"((?:[^"\\]|\\.)*)"', expr)
    if m:
        return m.group(1)
    return ""


def external_sources(mod_dir):
    """[(name, program argv, query expression)] of a module's data "external" blocks."""
    text = _module_text(mod_dir)
    out = []
    for m in re.finditer(r'^data\s+"external"\s+"(\w+)"\s*\{', text, re.M):
        body = _braced(text, m.end() - 1)
        prog = re.search(r"program\s*=\s*\[([^\]]*)\]", body)
        argv = [s.replace("${path.module}", mod_dir) for s in re.findall(r'"([^"]*)"', prog.group(1))] if prog else []
        q = re.search(r"^  query\s*=\s*", body, re.M)
        qexpr = ""
        if q:
            rest = body[q.end():]
            qexpr = "{" + _braced(rest, 0) + "}" if rest.startswith("{") else rest.split("\n", 1)[0]
        out.append((m.group(1), argv, qexpr))
    return out


def evaluate_query(mod_dir, qexpr, inputs):
    text = _module_text(mod_dir)
    local_exprs, defaults = _locals(text), _var_defaults(text)
    m = re.fullmatch(r"\s*local\.(\w+)\s*", qexpr)
    if m:
        qexpr = local_exprs.get(m.group(1), "")
    return {k: _value(e, inputs, defaults, local_exprs)
            for k, e in re.findall(r"^\s*(\w+)\s*=\s*([^\n]+?)\s*$", qexpr, re.M)}


def data_outputs(mod_dir):
    """{module output: (data source name, result key)} for outputs that read a data source."""
    out = {}
    text = _module_text(mod_dir)
    for m in re.finditer(r'^output\s+"(\w+)"\s*\{', text, re.M):
        v = re.search(r'value\s*=\s*data\.external\.(\w+)\.result(?:\["(\w+)"\]|\.(\w+))', _braced(text, m.end() - 1))
        if v:
            out[m.group(1)] = (v.group(1), v.group(2) or v.group(3))
    return out


def module_deps(block):
    return set(re.findall(r"\$\{module\.([A-Za-z0-9_.-]+?)\.", json.dumps(block)))


def refresh(doc, keys, root_vars, known_outputs):
    """Read the data sources of ``keys`` (and what they depend on) in dependency order.
    Returns ``(outputs by "<key>__<out>", error)``."""
    modules = doc.get("module") or {}
    want, todo = set(), list(keys)
    while todo:
        k = todo.pop()
        if k in modules and k not in want:
            want.add(k)
            todo.extend(module_deps(modules[k]))
    outs = dict(known_outputs)
    done = set()

    def sub(v):
        if isinstance(v, str):
            v = re.sub(r"\$\{var\.(\w+)\}", lambda m: str(root_vars.get(m.group(1), "")), v)
            return re.sub(r"\$\{module\.([A-Za-z0-9_.-]+?)\.(\w+)\}",
                          lambda m: str(outs.get(f"{m.group(1)}__{m.group(2)}", "")), v)
        if isinstance(v, dict):
            return {k: sub(x) for k, x in v.items()}
        if isinstance(v, list):
            return [sub(x) for x in v]
        return v

    while len(done) < len(want):
        ready = sorted(k for k in want - done if not (module_deps(modules[k]) & want) - done)
        if not ready:
            return outs, "Cycle in module references"
        for key in ready:
            done.add(key)
            d = local_dir(str(modules[key].get("source", "")))
            if d is None:
                continue
            inputs = sub(modules[key])
            results = {}
            for name, argv, qexpr in external_sources(d):
                query = evaluate_query(d, qexpr, inputs)
                bad_q = sorted(k for k, v in (query or {}).items() if not isinstance(v, str))
                if bad_q:  # the external data source's query is a map of strings
                    return outs, (f"Incorrect attribute value type\n\n  with module.{key}.data.external.{name}: "
                                  f"inappropriate value for attribute \"query\": element {bad_q[0]!r}: string required")
                try:
                    proc = subprocess.run(argv, input=json.dumps(query), capture_output=True,
                                                        text=True, timeout=120)
                except Exception as exc:  # noqa: BLE001
                    return outs, f"External Program Execution Failed\n\n  with module.{key}.data.external.{name}: {exc}"
                if proc.returncode != 0:
                    return outs, (f"External Program Execution Failed\n\n  with module.{key}.data.external.{name}\n\n"
                                  f"The data source received an unexpected error while attempting to execute the "
                                  f"program.\n\nProgram: {argv[-1]}\nError Message: {proc.stderr.strip()}\n"
                                  f"State: exit status {proc.returncode}")
                try:
                    results[name] = json.loads(proc.stdout)
                except ValueError:
                    return outs, f"Unexpected External Program Results\n\n  with module.{key}.data.external.{name}"
                res = results[name]
                if not isinstance(res, dict) or any(not isinstance(v, str) for v in res.values()):
                    # what Terraform's external data source accepts: a flat JSON object of strings
                    return outs, (f"Unexpected External Program Results\n\n  with module.{key}.data.external.{name}\n\n"
                                  "The data source received unexpected results after executing the program.\n\n"
                                  "Program output must be a JSON encoded map of string keys and string values.")
            for out, (src, field) in data_outputs(d).items():
                if src in results:
                    outs[f"{key}__{out}"] = str(results[src].get(field, ""))
    return outs, None


# --- bare-metal hosts (FAKE_TF_HOSTS) ------------------------------------------------------------

HOST_CONNECTION = "var/lib/rancher/agent/rancher2_connection_info.json"


def host_module(mod_dir):
    text = _module_text(mod_dir)
    return ('variable "host"' in text and 'variable "rancher_cluster_registration_token"' in text
            and "host        = var.host" in text)


def host_root(host):
    return os.path.join(os.environ["FAKE_TF_HOSTS"], host, "root")


def join_identity(doc_path, block):
    m = re.search(r"\$\{module\.([^.}]+)\.", str(block.get("rancher_cluster_registration_token", "")))
    return f"{os.path.abspath(doc_path)}:{m.group(1) if m else block.get('rancher_cluster_registration_token')}"


def join_host(key, block, path):
    """The host's side of an applied host module: ``None``, or the provisioner error."""
    host = str(block.get("host", ""))
    rec_path = os.path.join(host_root(host), HOST_CONNECTION)
    ident = join_identity(path, block)
    if os.path.exists(rec_path):
        prev = json.load(open(rec_path, encoding="utf-8"))
        if prev.get("cluster") != ident:
            return (f"remote-exec provisioner error\n\n  with module.{key}.terraform_data.install\n\n"
                    f"error executing \"/tmp/terraform_1.sh\": Process exited with status 1\n"
                    f"system-agent-install: rancher-system-agent is already installed on this host and connected "
                    f"to {prev.get('cluster')}: the node cannot join another cluster until it is uninstalled")
    os.makedirs(os.path.dirname(rec_path), exist_ok=True)
    with open(rec_path, "w", encoding="utf-8") as fh:
        json.dump({"cluster": ident, "module": key}, fh)
    return None


def _bracketed(text, start):
    """The text between the bracket at ``start`` and its match (strings skipped)."""
    depth, i, quote = 0, start, False
    while i < len(text):
        ch = text[i]
        if quote:
            if ch == "\\":
                i += 1
            elif ch == '"':
                quote = False
        elif ch == '"':
            quote = True
        elif ch in "[(":
            depth += 1
        elif ch in "])":
            depth -= 1
            if depth == 0:
                return text[start + 1:i]
        i += 1
    return text[start + 1:]


def destroy_provisioners(mod_dir):
    """The destroy-time remote-exec provisioners of the module's resources:
    ``[(count gate variable or None, {input key: variable}, inline parts, on_failure
    continue)]``; an inline part is ``("str", text)`` or ``("file", path)``."""
    text = _module_text(mod_dir)
    out = []
    for m in re.finditer(r'^resource\s+"\w+"\s+"\w+"\s*\{', text, re.M):
        body = _braced(text, m.end() - 1)
        gate = re.search(r"^\s*count\s*=\s*var\.(\w+)\s*\?\s*1\s*:\s*0\s*$", body, re.M)
        inp = re.search(r"^\s*input\s*=\s*\{", body, re.M)
        inputs = dict(re.findall(r"^\s*(\w+)\s*=\s*var\.(\w+)\s*$", _braced(body, inp.end() - 1), re.M)) if inp else {}
        for p in re.finditer(r'provisioner\s+"remote-exec"\s*\{', body):
            pb = _braced(body, p.end() - 1)
            if not re.search(r"^\s*when\s*=\s*destroy\s*$", pb, re.M):
                continue
            cont = re.search(r"^\s*on_failure\s*=\s*continue\s*$", pb, re.M) is not None
            il = re.search(r"\binline\s*=\s*\[", pb)
            if not il:
                continue
            parts = []
            for e in re.finditer(r'file\("\$\{path\.module\}/([^"]+)"\)|"((?:[^"\\]|\\.)*)"',
                                 _bracketed(pb, il.end() - 1)):
                parts.append(("file", os.path.join(mod_dir, e.group(1))) if e.group(1) else ("str", e.group(2)))
            out.append((gate.group(1) if gate else None, inputs, parts, cont))
    return out


def module_vars(block, mod_dir):
    """The module's variable values as applied: the block's arguments over the defaults
    (strings, as Terraform interpolates them: ``true`` / ``false`` for bools)."""
    vals = dict(_var_defaults(_module_text(mod_dir)))
    for k, v in block.items():
        vals[k] = ("true" if v else "false") if isinstance(v, bool) else v if isinstance(v, str) else json.dumps(v)
    return vals


def _falsy(v):
    return str(v).lower() in ("false", "0")


def run_destroy_provisioner(key, applied, inputs, parts, cont):
    """One destroy-time remote-exec against the host root, ``self`` being the resource as
    last applied (``applied``: the module's variable values then).  Terraform writes the
    ``inline`` parts, joined by newlines, to one script and runs it."""
    self_input = {k: applied.get(v, "") for k, v in inputs.items()}
    lines = []
    for kind, val in parts:
        if kind == "file":
            lines.append(open(val, encoding="utf-8").read())
        else:
            lines.append(re.sub(r"\$\{self\.input\.(\w+)\}", lambda m: str(self_input.get(m.group(1), "")),
                                val.encode().decode("unicode_escape")))
    env = dict(os.environ, TK_HOST_ROOT=host_root(str(applied.get("host", ""))))
    proc = subprocess.run(["bash", "-s"], input="\n".join(lines), env=env, capture_output=True, text=True,
                          timeout=120)
    sys.stdout.write(f"module.{key}: Destroying... (remote-exec)\n{proc.stdout}")
    if proc.returncode != 0:
        if not cont:
            return f"remote-exec provisioner error (destroy) in module.{key}: exit {proc.returncode}"
        sys.stderr.write(f"Warning: module.{key}: destroy-time provisioner failed (on_failure = continue): "
                         f"{proc.stderr[-300:]}\n")
    return None


def destroy_host(key, applied, mod_dir):
    """Run the destroy-time provisioners of a host module against its host root."""
    for gate, inputs, parts, cont in destroy_provisioners(mod_dir):
        if gate is not None and _falsy(applied.get(gate, "true")):
            continue  # count = 0: the resource (and its provisioner) does not exist
        err = run_destroy_provisioner(key, applied, inputs, parts, cont)
        if err:
            return err
    return None


def reapply_host(key, prior_vars, applied, mod_dir):
    """An apply of a host module already in the state: a count-gated resource whose count
    goes 1 -> 0 is destroyed, its destroy-time provisioner running (``self``: the resource
    as last applied).  Other argument changes update in place."""
    for gate, inputs, parts, cont in destroy_provisioners(mod_dir):
        if gate is not None and not _falsy(prior_vars.get(gate, "true")) and _falsy(applied.get(gate, "true")):
            err = run_destroy_provisioner(key, prior_vars, inputs, parts, cont)
            if err:
                return err
    return None


def applied_vars(st, key):
    for r in st.get("resources", []):
        if r.get("module") == f"module.{key}":
            return ((r.get("instances") or [{}])[0].get("attributes") or {}).get("tk_vars")
    return None


def root_variables(doc, argv):
    """Root variable values: declared defaults, then -var=name=value.  ``(values, error)``."""
    declared = doc.get("variable") or {}
    vals = {k: (v or {}).get("default", "") for k, v in declared.items()}
    for a in argv:
        if a.startswith("-var="):
            name, _, value = a[len("-var="):].partition("=")
            if name not in declared:
                return vals, (f'Value for undeclared variable\n\nA variable named "{name}" was assigned on the '
                              "command line, but the root module does not declare a variable of that name.")
            vals[name] = value
    return vals, None


def main() -> int:
    argv = sys.argv[1:]
    cmd = argv[0] if argv else ""
    version_s = os.environ.get("FAKE_TF_VERSION", "1.5.7")
    version = vtuple(version_s)
    doc = {}
    if os.path.exists("main.tf.json"):
        with open("main.tf.json", "r", encoding="utf-8") as fh:
            doc = json.load(fh)
    path = state_path(doc)
    prior = load_state(path) if doc else {}
    log = os.environ.get("FAKE_TF_LOG")
    if log:
        with open(log, "a", encoding="utf-8") as fh:
            fh.write(json.dumps({"argv": argv, "cwd": os.getcwd(), "doc": doc,
                                 "prior": {"serial": prior.get("serial"), "lineage": prior.get("lineage"),
                                           "modules": state_modules(prior)}}) + "\n")
    if cmd == "version":
        print(f"Terraform v{version_s}\non linux_amd64")
        return 0

    if cmd == "init":
        backend = ((doc.get("terraform") or {}).get("backend") or {})
        for kind in backend:
            if version >= (1, 3, 0) and kind in REMOVED_BACKENDS_1_3:
                return fail(f'Unsupported backend type\n\nThere is no backend type named "{kind}".')
        for key, mod in (doc.get("module") or {}).items():
            source = str(mod.get("source", ""))
            scheme = re.match(r"^([A-Za-z0-9]+)::", source)
            if scheme and scheme.group(1) not in GETTER_SCHEMES:
                # go-getter's forced-getter syntax with a getter Terraform does not have
                return fail(f'Failed to download module\n\nCould not download module "{key}" source code from '
                            f'"{source}": download not supported for scheme \'{scheme.group(1)}\'.')
            d = local_dir(source)
            if d is None:
                continue
            if not os.path.isdir(d):
                return fail(f"Unreadable module directory\n\nmodule.{key}: {d} does not exist")
            for req in required_versions(d):
                if not satisfied(version, req):
                    return fail(f"Unsupported Terraform Core version\n\n  on {d}/versions.tf:\n"
                                f"Module module.{key} requires Terraform {req}; this is {version_s}.")
        if os.environ.get("FAKE_TF_FAIL") == "init":
            return fail("fake failure of init")
        print("Terraform has been successfully initialized!")
        return 0

    if cmd in ("apply", "destroy", "output", "plan"):
        problem = validate(doc, version)
        if problem:
            return fail(problem)

    read = {}  # "<key>__<out>" values the data sources returned in this run's refresh
    if cmd in ("apply", "destroy", "plan"):
        root_vars, problem = root_variables(doc, argv)
        if problem:
            return fail(problem)
        if os.environ.get("FAKE_TF_EXTERNAL") == "1" and "-refresh=false" not in argv:
            targets = [a.split("=", 1)[1][len("module."):] for a in argv if a.startswith("-target=module.")]
            keys = targets if (cmd == "destroy" and targets) else list(doc.get("module") or {})
            if cmd == "destroy" and not targets:
                keys = [k for k in keys if k in state_modules(prior)]
            known = {k: v.get("value") for k, v in (prior.get("outputs") or {}).items()}
            read, problem = refresh(doc, keys, root_vars, known)
            if problem:
                return fail(problem)

    if cmd == "apply":
        st = prior or {"version": 4, "lineage": str(uuid.uuid4()), "serial": 0, "resources": [], "outputs": {}}
        st["terraform_version"] = version_s
        have = set(state_modules(st))
        new = [k for k in (doc.get("module") or {}) if k not in have]
        failing = os.environ.get("FAKE_TF_FAIL") == "apply"
        if failing:
            new = new[: len(new) // 2]
        refused = []
        if os.environ.get("FAKE_TF_HOSTS"):
            for key in list(new):
                block = (doc.get("module") or {})[key]
                d = local_dir(str(block.get("source", "")))
                if d and host_module(d):
                    err = join_host(key, block, path)
                    if err:
                        refused.append(err)
                        new.remove(key)
        if os.environ.get("FAKE_TF_HOSTS") and not failing:
            for key in sorted(have & set(doc.get("module") or {})):
                block = (doc.get("module") or {})[key]
                d = local_dir(str(block.get("source", "")))
                prior_vars = applied_vars(st, key)
                if d and host_module(d) and prior_vars is not None:
                    now = module_vars(block, d)
                    err = reapply_host(key, prior_vars, now, d)
                    if err:
                        refused.append(err)
                        continue
                    for r in st["resources"]:
                        if r.get("module") == f"module.{key}":
                            r["instances"][0]["attributes"]["tk_vars"] = now  # updated in place
        for key in new:
            attrs = {"id": str(uuid.uuid4())}
            block = (doc.get("module") or {})[key]
            d = local_dir(str(block.get("source", "")))
            if d and os.path.isdir(d):
                attrs["tk_vars"] = module_vars(block, d)
            st["resources"].append({"module": f"module.{key}", "mode": "managed", "type": "terraform_data",
                                    "name": "fake", "instances": [{"attributes": attrs}]})
        done = set(state_modules(st))
        outs = {}
        for name, spec in (doc.get("output") or {}).items():
            m = re.fullmatch(r"\$\{module\.([^.}]+)\.[^}]+\}", str(spec.get("value", "")))
            if m and m.group(1) not in done:
                continue
            value = read.get(name) or (prior.get("outputs") or {}).get(name, {}).get("value") or f"fake-{name}"
            outs[name] = {"value": value, "type": "string", "sensitive": bool(spec.get("sensitive"))}
        st["outputs"] = outs
        st["serial"] = int(st.get("serial", 0)) + 1
        save_state(path, st)
        if failing:
            return fail("fake failure of apply")
        if refused:
            return fail("\n\nError: ".join(refused))
        print(f"Apply complete! Resources: {len(new)} added, 0 changed, 0 destroyed.")
        return 0

    if cmd == "destroy":
        if os.environ.get("FAKE_TF_FAIL") == "destroy":
            return fail("fake failure of destroy")
        targets = [a.split("=", 1)[1] for a in argv if a.startswith("-target=")]
        st = prior or {"version": 4, "lineage": str(uuid.uuid4()), "serial": 0, "resources": [], "outputs": {}}
        gone = {t[len("module."):] for t in targets} if targets else set(state_modules(st))
        if os.environ.get("FAKE_TF_HOSTS"):
            for key in sorted(gone & set(state_modules(st))):
                block = (doc.get("module") or {}).get(key) or {}
                d = local_dir(str(block.get("source", "")))
                if d and host_module(d):
                    # self: the resource as last applied (the current configuration's values
                    # only for a state written before they were recorded)
                    err = destroy_host(key, applied_vars(st, key) or module_vars(block, d), d)
                    if err:
                        return fail(err)
        st["resources"] = [r for r in st.get("resources", []) if r.get("module", "")[len("module."):] not in gone]
        st["outputs"] = {k: v for k, v in (st.get("outputs") or {}).items()
                         if not any(k.startswith(g + "__") for g in gone)}
        st["serial"] = int(st.get("serial", 0)) + 1
        save_state(path, st)
        print(f"Destroy complete! Resources: {len(gone)} destroyed.")
        return 0

    if cmd == "output":
        outs = prior.get("outputs", {})
        module = next((a.split("=", 1)[1] for a in argv if a.startswith("-module=")), None)
        if module is None and "-module" in argv:
            module = argv[argv.index("-module") + 1]
        if module:
            outs = {k[len(module) + 2:]: v for k, v in outs.items() if k.startswith(module + "__")}
        if "-json" in argv:
            print(json.dumps(outs))
        else:
            for k in sorted(outs):
                print(f"{k} = " + ("<sensitive>" if outs[k].get("sensitive") else str(outs[k]["value"])))
        return 0
    return 0


if __name__ == "__main__":
    sys.exit(main())
