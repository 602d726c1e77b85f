"""Process execution (reference ``shell/run_shell_cmd.go:8-29``).

``run_shell_command`` inherits stdin/stdout/stderr like the reference.  Added:
an optional timeout and a hook so tests can swap in a recorder.
"""

import os
import shutil
import subprocess
from dataclasses import dataclass
from typing import Dict, List, Optional

from ..errors import ExecutorError


@dataclass
class ShellOptions:
    working_dir: Optional[str] = None
    env: Optional[Dict[str, str]] = None
    timeout: Optional[float] = None
    capture: bool = False


@dataclass
class ShellResult:
    returncode: int
    stdout: str = ""
    stderr: str = ""


def run_shell_command(options: Optional[ShellOptions], command: str, *args: str) -> ShellResult:
    opts = options or ShellOptions()
    exe = shutil.which(command, path=(opts.env or os.environ).get("PATH")) if os.sep not in command else command
    if exe is None:
        raise ExecutorError(f'exec: "{command}": executable file not found in $PATH')
    env = dict(os.environ)
    if opts.env:
        env.update(opts.env)
    try:
        proc = subprocess.run(
            [exe, *args], cwd=opts.working_dir, env=env, timeout=opts.timeout,
            capture_output=opts.capture, text=opts.capture, check=False,
        )
    except subprocess.TimeoutExpired as exc:
        raise ExecutorError(f"{command} {' '.join(args)}: timed out after {opts.timeout}s") from exc
    except OSError as exc:  # a path that is not there, or not executable (Go: fork/exec <path>: ...)
        raise ExecutorError(f"fork/exec {exe}: {exc.strerror or exc}") from exc
    if proc.returncode != 0:
        raise ExecutorError(f"exit status {proc.returncode}")
    return ShellResult(proc.returncode, proc.stdout or "", proc.stderr or "")


def capture_command(command: str, *args: str, working_dir: Optional[str] = None,
                    env: Optional[Dict[str, str]] = None, timeout: Optional[float] = 60) -> ShellResult:
    return run_shell_command(ShellOptions(working_dir=working_dir, env=env, timeout=timeout, capture=True),
                             command, *args)


def which(command: str, env: Optional[Dict[str, str]] = None) -> Optional[str]:
    return shutil.which(command, path=(env or os.environ).get("PATH"))


__all__: List[str] = ["ShellOptions", "ShellResult", "run_shell_command", "capture_command", "which"]
