"""Interactive prompt interface (the reference's promptui usage).

Workflows never talk to a terminal directly; they call a :class:`Prompter`.
Implementations:

* :class:`TerminalPrompter` — numbered-menu prompts on stdin/stdout (promptui
  replacement: ``Select``, ``Prompt`` with default/validate/mask, ``SelectWithAdd``,
  searchable selects, Yes/No confirmation of ``util/confirm_prompt.go:10-35``);
* :class:`ScriptedPrompter` — deterministic answers for tests (the reference had
  no way to test interactive paths);
* :class:`NoPrompter` — raises if a prompt is reached (non-interactive safety net).
"""

import getpass
import sys
from typing import Any, Callable, List, Optional, Sequence, Tuple

from ..errors import PromptAborted, TKError

Validator = Optional[Callable[[str], Optional[str]]]
"""A validator returns an error message (invalid) or ``None`` (valid)."""


class Prompter:
    def select(self, label: str, items: Sequence[str], searchable: bool = False) -> Tuple[int, str]:
        raise NotImplementedError

    def prompt(self, label: str, default: Optional[str] = None, validate: Validator = None, mask: bool = False) -> str:
        raise NotImplementedError

    def select_with_add(self, label: str, items: Sequence[str], add_label: str) -> Tuple[int, str]:
        """Select from ``items`` or return ``(-1, <new value>)`` (promptui ``SelectWithAdd``)."""
        raise NotImplementedError

    def confirm(self, label: str, selected: str = "") -> bool:
        idx, _ = self.select(label, ["Yes", "No"])
        return idx == 0

    def yes_no(self, label: str) -> bool:
        idx, _ = self.select(label, ["Yes", "No"])
        return idx == 0


class NoPrompter(Prompter):
    def _fail(self, label: str):
        raise TKError(f"interactive prompt '{label}' reached in non-interactive mode")

    def select(self, label, items, searchable=False):
        self._fail(label)

    def prompt(self, label, default=None, validate=None, mask=False):
        self._fail(label)

    def select_with_add(self, label, items, add_label):
        self._fail(label)


class TerminalPrompter(Prompter):
    def __init__(self, stdin=None, stdout=None):
        self.stdin = stdin or sys.stdin
        self.stdout = stdout or sys.stdout

    def _readline(self, mask: bool = False) -> str:
        if mask and self.stdin is sys.stdin and sys.stdin.isatty():
            try:
                return getpass.getpass("")
            except (EOFError, KeyboardInterrupt) as exc:
                raise PromptAborted("^C") from exc
        try:
            line = self.stdin.readline()
        except KeyboardInterrupt as exc:
            raise PromptAborted("^C") from exc
        if line == "":
            raise PromptAborted("EOF")
        return line.rstrip("\n")

    def _write(self, text: str) -> None:
        self.stdout.write(text)
        self.stdout.flush()

    def select(self, label, items, searchable=False):
        items = list(items)
        if not items:
            raise TKError(f"no choices available for '{label}'")
        shown = list(range(len(items)))
        while True:
            self._write(f"{label}?\n")
            for n, i in enumerate(shown, 1):
                self._write(f"  {n}) {items[i]}\n")
            hint = " (number" + (", or text to filter" if searchable else "") + "): "
            self._write(hint)
            answer = self._readline().strip()
            if answer.isdigit() and 1 <= int(answer) <= len(shown):
                i = shown[int(answer) - 1]
                self._write(f"✔ {label}: {items[i]}\n")
                return i, items[i]
            if answer in items:
                i = items.index(answer)
                return i, items[i]
            if searchable and answer:
                needle = answer.lower().replace(" ", "")
                filtered = [i for i in range(len(items)) if needle in items[i].lower().replace(" ", "")]
                if filtered:
                    shown = filtered
                    continue
            self._write("invalid choice\n")

    def prompt(self, label, default=None, validate=None, mask=False):
        while True:
            suffix = f" [{default}]" if default not in (None, "") else ""
            self._write(f"{label}{suffix}: ")
            answer = self._readline(mask=mask)
            if answer == "" and default is not None:
                answer = default
            err = validate(answer) if validate else None
            if err:
                self._write(f"✗ {err}\n")
                continue
            return answer

    def select_with_add(self, label, items, add_label):
        idx, value = self.select(label, list(items) + [add_label])
        if idx == len(items):
            return -1, self.prompt(add_label)
        return idx, value


class ScriptedPrompter(Prompter):
    """Answers prompts from a queue; records every question for assertions.

    Each answer is either a string (matched against select items, or typed into
    a prompt; ``""`` means "accept the default") or an int (select index).
    """

    def __init__(self, answers: Sequence[Any] = ()):
        self.answers: List[Any] = list(answers)
        self.asked: List[Tuple[str, str]] = []

    def _next(self, kind: str, label: str):
        self.asked.append((kind, label))
        if not self.answers:
            raise PromptAborted(f"no scripted answer for {kind} '{label}'")
        return self.answers.pop(0)

    def select(self, label, items, searchable=False):
        items = list(items)
        ans = self._next("select", label)
        if isinstance(ans, int) and not isinstance(ans, bool):
            return ans, items[ans]
        if ans in items:
            return items.index(ans), ans
        lowered = [i.lower() for i in items]
        if str(ans).lower() in lowered:
            i = lowered.index(str(ans).lower())
            return i, items[i]
        raise PromptAborted(f"scripted answer {ans!r} not in choices {items} for '{label}'")

    def prompt(self, label, default=None, validate=None, mask=False):
        ans = self._next("prompt", label)
        ans = default if (ans == "" and default is not None) else str(ans)
        err = validate(ans) if validate else None
        if err:
            raise TKError(err)
        return ans

    def select_with_add(self, label, items, add_label):
        items = list(items)
        ans = self._next("select_with_add", label)
        if isinstance(ans, tuple) and ans and ans[0] == "add":
            return -1, ans[1]
        if isinstance(ans, int) and not isinstance(ans, bool):
            return ans, items[ans]
        if ans in items:
            return items.index(ans), ans
        return -1, str(ans)
