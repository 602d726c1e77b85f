"""Host transports used by the DirectExecutor's fan-out.

===================  =============================================================
``ssh`` (default)    ``ssh``/``scp`` subprocesses with connection multiplexing
                     (ControlMaster) and an optional hop through the bastion —
                     Terraform's ``remote-exec`` equivalent (T16), which in the
                     reference ignores the bastion for managers (Q11).  Host keys
                     are checked against the manager's pinned keys
                     (``parallel/hostkeys.py``, bound by the executor): trust on
                     first use, a changed key refused
``agent``            HTTPS to a ``tk-node-agent`` (``agent+https://host:port``
                     host strings; ``agent+http://`` on loopback only); the agent
                     runs plan steps natively
``local``            runs the rendered script with ``bash`` on this machine
                     (single-box development)
``recording``        test double: records plans/scripts, scripted failures
===================  =============================================================

Every transport returns the same result document for a plan:
``{"hostname", "ok", "error", "ms", "steps": [{name, ok, ms}], "labels", ...}``.
"""

import os
import shlex
import subprocess
import tempfile
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..cloud.http import HTTPClient
from ..errors import ExecutorError
from ..node.cleanup import cleanup_script, parse_cleanup_markers
from ..node.plan import BootstrapPlan, parse_step_markers


def _cleanup_result(rc: int, stdout: str, stderr: str, where: str) -> Dict[str, Any]:
    """A cleanup script's run -> its report (``node/cleanup.py`` markers); an exit without
    the final marker (unreachable host: ssh's 255) is an error."""
    rep = parse_cleanup_markers(stdout)
    if not rep["complete"]:
        rep.update(ok=False, error=f"{where}: exit {rc}: {(stderr or stdout)[-500:]}")
    elif rc != 0:
        failed = [a["what"] for a in rep["actions"] if a["status"] == "failed"]
        rep["error"] = f"{where}: failed: {', '.join(failed) or 'exit ' + str(rc)}"
    return rep


@dataclass
class HostRef:
    address: str
    ssh_user: str = "ubuntu"
    key_path: str = "~/.ssh/id_rsa"
    bastion_host: str = ""
    bastion_user: str = ""

    @property
    def scheme(self) -> str:
        if self.address.startswith("agent+"):
            return "agent"
        if self.address in ("local", "localhost-exec"):
            return "local"
        return "ssh"

    @property
    def agent_url(self) -> str:
        return self.address[len("agent+"):]


class Transport:
    name = "abstract"

    def bind_host_keys(self, keys: Any) -> None:
        """Use ``keys`` (:class:`~.hostkeys.HostKeys`) for SSH host-key checks from now on."""

    def run_plan(self, host: HostRef, plan: BootstrapPlan, timeout: float = 3600) -> Dict[str, Any]:
        raise NotImplementedError

    def run_script(self, host: HostRef, script: str, timeout: float = 3600) -> str:
        raise NotImplementedError

    def put_file(self, host: HostRef, local_path: str, remote_path: str, mode: int = 0o755) -> None:
        raise NotImplementedError

    def cleanup_host(self, host: HostRef, timeout: float = 600) -> Dict[str, Any]:
        """Take the host out of its cluster (``node/cleanup.py``): ``{"ok", "actions"}``,
        plus ``"error"`` when the host could not be reached or the cleanup not run."""
        raise NotImplementedError

    def spawn(self, host: HostRef, script: str) -> subprocess.Popen:
        """Start ``bash -c script`` on the host and return at once; stdout is a text pipe the
        caller reads while it runs (the process-mode RCCL gate needs rank 0's first line
        before the other nodes can start).  stdin is a pipe the caller closes when done:
        the script may watch it to learn that its caller went away."""
        raise NotImplementedError


def _shell_result(plan: BootstrapPlan, output: str, rc: int, ms: float, err: str = "") -> Dict[str, Any]:
    markers = parse_step_markers(output + "\n" + err)
    steps = [{"name": n, "ok": m["status"] == "ok", "ms": m["ms"]} for n, m in markers.items()
             if m["status"] != "start"]
    failed = [n for n, m in markers.items() if m["status"] == "failed"]
    ok = rc == 0 and "::tk-done" in output
    return {"hostname": plan.hostname, "ok": ok, "ms": ms, "steps": steps,
            "error": None if ok else f"step {failed[0] if failed else '?'} failed (rc={rc}): {err[-800:]}",
            "labels": {}, "capacity": {}}


class SSHTransport(Transport):
    name = "ssh"

    def __init__(self, strict_host_keys: bool = False, connect_timeout: int = 15, control_dir: Optional[str] = None,
                 extra_opts: Optional[List[str]] = None, host_keys: Any = None):
        # strict_host_keys: only hosts already in the user's own known_hosts (ssh's default
        # files, StrictHostKeyChecking=yes).  Otherwise the manager's pinned keys when the
        # executor bound them (bind_host_keys), else a private known_hosts for this
        # transport's lifetime: either way trust on first use, a changed key refused.
        self.strict = strict_host_keys
        self.connect_timeout = connect_timeout
        self.control_dir = control_dir or tempfile.mkdtemp(prefix="tk-ssh-")
        self.extra = list(extra_opts or [])
        self.host_keys = host_keys

    def bind_host_keys(self, keys: Any) -> None:
        self.host_keys = keys

    def _key_opts(self) -> List[str]:
        if self.strict:
            return ["-o", "StrictHostKeyChecking=yes"]
        if self.host_keys is not None:
            return self.host_keys.ssh_options()
        from .hostkeys import NEGOTIATION_OPTS

        return ["-o", f"UserKnownHostsFile={self.control_dir}/known_hosts", "-o", "StrictHostKeyChecking=accept-new",
                "-o", "HashKnownHosts=no", "-o", "GlobalKnownHostsFile=/dev/null", *NEGOTIATION_OPTS]

    def base_opts(self, host: HostRef) -> List[str]:
        opts = ["-o", "BatchMode=yes", "-o", f"ConnectTimeout={self.connect_timeout}",
                "-o", "ControlMaster=auto", "-o", f"ControlPath={self.control_dir}/%C",
                "-o", "ControlPersist=120s", "-o", "ServerAliveInterval=15", "-o", "LogLevel=ERROR"]
        keys = self._key_opts()
        opts += keys
        key = ["-i", os.path.expanduser(host.key_path)] if host.key_path else []
        opts += key
        if host.bastion_host:
            # the hop checks the bastion's key the same way (-J would not pass these options on)
            user = host.bastion_user or host.ssh_user
            hop = ["ssh", "-o", "BatchMode=yes", "-o", f"ConnectTimeout={self.connect_timeout}", *keys, *key,
                   "-W", "%h:%p", f"{user}@{host.bastion_host}"]
            opts += ["-o", "ProxyCommand=" + " ".join(shlex.quote(a) for a in hop)]
        return opts + self.extra

    def _check_key(self, host: HostRef, rc: int, stderr: str) -> None:
        from .hostkeys import looks_like_mismatch, mismatch_error

        if rc == 255 and looks_like_mismatch(stderr or ""):
            manager = getattr(self.host_keys, "manager", "")
            raise mismatch_error(host.address if host.address in stderr or not host.bastion_host
                                 else f"{host.address} (or its bastion {host.bastion_host})", stderr, manager)

    def ssh_argv(self, host: HostRef, remote_cmd: str) -> List[str]:
        return ["ssh", *self.base_opts(host), f"{host.ssh_user}@{host.address}", remote_cmd]

    def run_script(self, host: HostRef, script: str, timeout: float = 3600) -> str:
        proc = subprocess.run(self.ssh_argv(host, "bash -s"), input=script, capture_output=True, text=True,
                              timeout=timeout, check=False)
        self._check_key(host, proc.returncode, proc.stderr)
        if proc.returncode != 0:
            raise ExecutorError(f"ssh {host.ssh_user}@{host.address}: exit {proc.returncode}: "
                                f"{proc.stderr[-800:]}")
        return proc.stdout

    def run_plan(self, host: HostRef, plan: BootstrapPlan, timeout: float = 3600) -> Dict[str, Any]:
        t0 = time.perf_counter()
        proc = subprocess.run(self.ssh_argv(host, "bash -s"), input=plan.render_shell(), capture_output=True,
                              text=True, timeout=timeout, check=False)
        self._check_key(host, proc.returncode, proc.stderr)
        return _shell_result(plan, proc.stdout, proc.returncode, (time.perf_counter() - t0) * 1e3, proc.stderr)

    def cleanup_host(self, host: HostRef, timeout: float = 600) -> Dict[str, Any]:
        proc = subprocess.run(self.ssh_argv(host, "bash -s"), input=cleanup_script(), capture_output=True,
                              text=True, timeout=timeout, check=False)
        self._check_key(host, proc.returncode, proc.stderr)
        return _cleanup_result(proc.returncode, proc.stdout, proc.stderr, f"ssh {host.ssh_user}@{host.address}")

    def put_file(self, host: HostRef, local_path: str, remote_path: str, mode: int = 0o755) -> None:
        dirname = os.path.dirname(remote_path)
        self.run_script(host, f"sudo mkdir -p {shlex.quote(dirname)} && sudo chown \"$(id -un)\" "
                              f"{shlex.quote(dirname)}\n")
        proc = subprocess.run(["scp", "-q", *self.base_opts(host), local_path,
                               f"{host.ssh_user}@{host.address}:{remote_path}"], capture_output=True, text=True,
                              check=False)
        self._check_key(host, proc.returncode, proc.stderr)
        if proc.returncode != 0:
            raise ExecutorError(f"scp {local_path} -> {host.address}:{remote_path}: {proc.stderr[-500:]}")
        self.run_script(host, f"chmod {mode:o} {shlex.quote(remote_path)}\n")

    def spawn(self, host: HostRef, script: str) -> subprocess.Popen:
        # stdin stays an open pipe: the remote side sees EOF when the caller closes it or
        # this ssh client dies (readiness/process_gate.py's node-side watchdog)
        return subprocess.Popen(self.ssh_argv(host, "bash -c " + shlex.quote(script)), stdin=subprocess.PIPE,
                                stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


class LocalTransport(Transport):
    """Runs scripts with the local ``bash`` (development / single-box)."""

    name = "local"

    def __init__(self, env: Optional[Dict[str, str]] = None):
        self.env = env

    def _env(self) -> Dict[str, str]:
        e = dict(os.environ)
        e.update(self.env or {})
        return e

    def run_script(self, host: HostRef, script: str, timeout: float = 3600) -> str:
        proc = subprocess.run(["bash", "-s"], input=script, capture_output=True, text=True, timeout=timeout,
                              env=self._env(), check=False)
        if proc.returncode != 0:
            raise ExecutorError(f"local script exit {proc.returncode}: {proc.stderr[-800:]}")
        return proc.stdout

    def run_plan(self, host: HostRef, plan: BootstrapPlan, timeout: float = 3600) -> Dict[str, Any]:
        t0 = time.perf_counter()
        proc = subprocess.run(["bash", "-s"], input=plan.render_shell(), capture_output=True, text=True,
                              timeout=timeout, env=self._env(), check=False)
        return _shell_result(plan, proc.stdout, proc.returncode, (time.perf_counter() - t0) * 1e3, proc.stderr)

    def cleanup_host(self, host: HostRef, timeout: float = 600) -> Dict[str, Any]:
        proc = subprocess.run(["bash", "-s"], input=cleanup_script(), capture_output=True, text=True,
                              timeout=timeout, env=self._env(), check=False)
        return _cleanup_result(proc.returncode, proc.stdout, proc.stderr, "local")

    def put_file(self, host: HostRef, local_path: str, remote_path: str, mode: int = 0o755) -> None:
        os.makedirs(os.path.dirname(remote_path), exist_ok=True)
        with open(local_path, "rb") as src, open(remote_path, "wb") as dst:
            dst.write(src.read())
        os.chmod(remote_path, mode)

    def spawn(self, host: HostRef, script: str) -> subprocess.Popen:
        return subprocess.Popen(["bash", "-c", script], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                stderr=subprocess.PIPE, text=True, env=self._env())


class AgentTransport(Transport):
    """HTTP(S) to node agents (``node/security.py``).  With ``pki`` (the cluster manager's
    agent CA + secret): each agent's token is derived for its address, ``https`` agents
    are verified against that CA only, and a plain ``http`` agent is refused unless it is
    on loopback.  Without ``pki`` (development, in-process tests): the shared ``token``
    (or ``tokens[url]``)."""

    name = "agent"

    def __init__(self, token: str = "", tokens: Optional[Dict[str, str]] = None, timeout: float = 3600,
                 pki: Any = None):
        self.token = token
        self.tokens = dict(tokens or {})
        self.timeout = timeout
        self.pki = pki
        self._ctx = pki.client_context() if pki is not None else None
        self._clients: Dict[str, HTTPClient] = {}
        self._mu = threading.Lock()

    def _client(self, host: HostRef) -> HTTPClient:
        url = host.agent_url
        with self._mu:
            c = self._clients.get(url)
            if c is None:
                if self.pki is not None:
                    from ..node.security import agent_address, is_loopback

                    addr = agent_address(url)
                    if not url.startswith("https://") and not is_loopback(addr):
                        raise ExecutorError(f"refusing plain HTTP to the node agent at {url}: agents off "
                                            "loopback serve TLS (agent+https://)")
                    tok = self.tokens.get(url) or self.pki.node_token(addr)
                else:
                    tok = self.tokens.get(url, self.token)
                c = HTTPClient(base_url=url, timeout=self.timeout, retries=1, ssl_context=self._ctx,
                               default_headers={"X-TK-Agent-Token": tok})
                self._clients[url] = c
            return c

    def run_plan(self, host: HostRef, plan: BootstrapPlan, timeout: float = 3600) -> Dict[str, Any]:
        return self._client(host).post_json("/v1/plan", {"plan": plan.to_json()})

    def post(self, host: HostRef, path: str, body: Dict[str, Any]) -> Dict[str, Any]:
        return self._client(host).post_json(path, body)

    def get(self, host: HostRef, path: str, params: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
        return self._client(host).request("GET", path, params=params).json()

    def run_script(self, host: HostRef, script: str, timeout: float = 3600) -> str:
        raise ExecutorError("the node agent does not execute shell scripts; use an agent plan or the ssh transport")

    def cleanup_host(self, host: HostRef, timeout: float = 600) -> Dict[str, Any]:
        # the agent's own fixed-argv teardown (NodeAgent.cleanup): no script crosses the wire
        try:
            return self._client(host).post_json("/v1/cleanup", {})
        except Exception as exc:  # noqa: BLE001 - reported, the destroy goes on
            return {"ok": False, "error": f"{host.agent_url}: {type(exc).__name__}: {exc}", "actions": []}

    def put_file(self, host: HostRef, local_path: str, remote_path: str, mode: int = 0o755) -> None:
        return None  # agents run the native probes in-process; nothing to upload


@dataclass
class RecordingTransport(Transport):
    """Test double: records every call; ``fail`` maps hostname -> error text."""

    fail: Dict[str, str] = field(default_factory=dict)
    delay: float = 0.0
    on_plan: Optional[Callable[[HostRef, BootstrapPlan], Dict[str, Any]]] = None
    name: str = "recording"

    def __post_init__(self):
        self.plans: List[BootstrapPlan] = []
        self.scripts: List[str] = []
        self.files: List[str] = []
        self.cleanups: List[str] = []
        self._mu = threading.Lock()

    def run_plan(self, host: HostRef, plan: BootstrapPlan, timeout: float = 3600) -> Dict[str, Any]:
        with self._mu:
            self.plans.append(plan)
        if self.delay:
            time.sleep(self.delay)
        if self.on_plan is not None:
            return self.on_plan(host, plan)
        if plan.hostname in self.fail:
            return {"hostname": plan.hostname, "ok": False, "error": self.fail[plan.hostname], "steps": []}
        return {"hostname": plan.hostname, "ok": True, "error": None, "ms": self.delay * 1e3,
                "steps": [{"name": s.name, "ok": True, "ms": 0} for s in plan.steps], "labels": {}, "capacity": {}}

    def run_script(self, host: HostRef, script: str, timeout: float = 3600) -> str:
        with self._mu:
            self.scripts.append(script)
        return ""

    def put_file(self, host: HostRef, local_path: str, remote_path: str, mode: int = 0o755) -> None:
        with self._mu:
            self.files.append(remote_path)

    def cleanup_host(self, host: HostRef, timeout: float = 600) -> Dict[str, Any]:
        with self._mu:
            self.cleanups.append(host.address)
        if host.address in self.fail:
            return {"ok": False, "error": self.fail[host.address], "actions": []}
        return {"ok": True, "actions": []}


class TransportRouter(Transport):
    """Dispatch by :attr:`HostRef.scheme`."""

    name = "router"

    def __init__(self, ssh: Optional[Transport] = None, agent: Optional[Transport] = None,
                 local: Optional[Transport] = None):
        self.routes = {"ssh": ssh or SSHTransport(), "agent": agent or AgentTransport(),
                       "local": local or LocalTransport()}

    def for_host(self, host: HostRef) -> Transport:
        return self.routes[host.scheme]

    def bind_host_keys(self, keys: Any) -> None:
        for t in self.routes.values():
            t.bind_host_keys(keys)

    def run_plan(self, host, plan, timeout=3600):
        return self.for_host(host).run_plan(host, plan, timeout)

    def run_script(self, host, script, timeout=3600):
        return self.for_host(host).run_script(host, script, timeout)

    def put_file(self, host, local_path, remote_path, mode=0o755):
        return self.for_host(host).put_file(host, local_path, remote_path, mode)

    def cleanup_host(self, host, timeout=600):
        return self.for_host(host).cleanup_host(host, timeout)

    def spawn(self, host, script):
        return self.for_host(host).spawn(host, script)
