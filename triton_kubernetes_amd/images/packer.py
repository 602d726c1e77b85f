"""YAML -> Packer JSON template renderer (reference ``packer/packer-config``, B4).

Behaviour kept from the reference tool:

* an ``!include <path>`` tag pulls in another YAML file, resolved relative to
  the file that contains the tag (absolute paths are used as is);
* a top-level ``variables`` list of mappings is merged into one mapping;
* lists-of-lists in ``builders`` / ``provisioners`` / ``post-processors`` are
  flattened, so one include can contribute several steps.

Differences (deliberate): parsing uses ``yaml.SafeLoader`` (the reference used
the full loader, which can construct arbitrary Python objects), include cycles
are an error instead of a recursion crash, and a missing template exits 2 with
a message instead of hitting the reference's ``std.stderr`` NameError
(``packer/packer-config:112``).

    python -m triton_kubernetes_amd.images mi355x-node.yaml > mi355x-node.json
"""

import json
import os
import sys
from typing import Any, Dict, List, Optional, Sequence, Tuple

import yaml

TEMPLATES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "templates")
FILES_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "files")
FLATTEN = ("builders", "provisioners", "post-processors")


class TemplateError(Exception):
    pass


def _make_loader(path: str, stack: Tuple[str, ...]):
    base = os.path.dirname(os.path.abspath(path))

    class IncludeLoader(yaml.SafeLoader):
        pass

    def include(loader: yaml.SafeLoader, node: yaml.Node) -> Any:
        rel = loader.construct_scalar(node)
        target = rel if os.path.isabs(rel) else os.path.join(base, rel)
        return _load(target, stack)

    IncludeLoader.add_constructor("!include", include)
    return IncludeLoader


def _load(path: str, stack: Tuple[str, ...] = ()) -> Any:
    real = os.path.realpath(path)
    if real in stack:
        chain = " -> ".join(os.path.basename(p) for p in stack + (real,))
        raise TemplateError(f"include cycle: {chain}")
    if not os.path.isfile(real):
        raise TemplateError(f"Template not found: {path}")
    with open(real, "r", encoding="utf-8") as fh:
        return yaml.load(fh, Loader=_make_loader(real, stack + (real,)))  # noqa: S506 - SafeLoader subclass


def load_template(path: str) -> Dict[str, Any]:
    doc = _load(path)
    if not isinstance(doc, dict):
        raise TemplateError(f"{path}: a template must be a mapping")
    variables = doc.get("variables")
    if isinstance(variables, list):
        merged: Dict[str, Any] = {}
        for entry in variables:
            if isinstance(entry, dict):
                merged.update(entry)
        doc["variables"] = merged
    for section in FLATTEN:
        items = doc.get(section)
        if items is None:
            continue
        flat: List[Any] = []
        for item in items:
            flat.extend(item if isinstance(item, list) else [item])
        doc[section] = flat
    return doc


def render_template(path: str, overrides: Optional[Dict[str, Any]] = None) -> str:
    """Packer JSON for ``path``; ``overrides`` replace entries of ``variables``."""
    doc = load_template(path)
    if overrides:
        doc.setdefault("variables", {}).update(overrides)
    variables = doc.get("variables")
    if isinstance(variables, dict) and "files_dir" in variables and not variables["files_dir"]:
        variables["files_dir"] = FILES_DIR
    return json.dumps(doc, indent=2, separators=(",", ": ")) + "\n"


def resolve(name: str) -> str:
    """A path as given, or the name of a bundled template."""
    if os.path.exists(name):
        return name
    for cand in (os.path.join(TEMPLATES_DIR, name), os.path.join(TEMPLATES_DIR, name + ".yaml")):
        if os.path.exists(cand):
            return cand
    return name


def main(argv: Optional[Sequence[str]] = None) -> int:
    args = list(sys.argv[1:] if argv is None else argv)
    if not args or args[0] in ("-h", "--help"):
        sys.stderr.write("usage: images <template.yaml|bundled-name> [var=value ...]\n")
        sys.stderr.write("bundled: " + ", ".join(sorted(f[:-5] for f in os.listdir(TEMPLATES_DIR)
                                                        if f.endswith(".yaml"))) + "\n")
        return 1
    overrides = {}
    for kv in args[1:]:
        k, sep, v = kv.partition("=")
        if not sep:
            sys.stderr.write(f"ERROR: expected var=value, got {kv!r}\n")
            return 1
        overrides[k] = v
    try:
        sys.stdout.write(render_template(resolve(args[0]), overrides))
    except TemplateError as exc:
        sys.stderr.write(f"ERROR: {exc}\n")
        return 2
    return 0
