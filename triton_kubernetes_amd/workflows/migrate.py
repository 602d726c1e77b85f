"""``migrate manager``: move a cluster manager's document onto this framework's modules.

A user switching from the reference has ``~/.triton-kubernetes/<manager>/main.tf.json``
(or the Manta copy) whose module blocks point at the reference's Terraform 0.11 modules
(``github.com/joyent/triton-kubernetes//terraform/modules/<name>?ref=master``,
``create/manager.go:160-171``).  Terraform >= 0.12 cannot parse those, and the reference
modules lack the MI355X host and add-on modules.  Module keys, variable names and the
backend block are compatible by design, so migration is a source rewrite plus a check:

1. every module block whose source is not this framework's source for that module (the
   location-free ``tk::terraform/modules/<m>?ref=v<version>`` of the packaged tree, or
   ``source_url``/``source_ref``) is pointed at it.  This also re-pins documents written
   by another version of this CLI (a ``tk::`` source with another ``ref``, which every
   executor refuses) and rewrites the absolute paths of one operator's install that
   documents of earlier versions persisted;
2. each rewritten block is checked against the new module the way ``terraform plan``
   would (``terraform/hcl.py:check_inputs``, then ``terraform/plan.py`` evaluates every
   expression of the module for the block's inputs): unknown arguments (dropped with
   ``migrate_drop_unknown: true``, else reported and the migration refused), missing
   required arguments (refused), failing validations (e.g. a Kubernetes release the
   pinned Rancher does not ship: reported as a warning, because the running cluster keeps
   its version until it is recreated);
3. the reference only created RKE1 clusters (v3 cluster + ``rancher-agent``), so a
   rewritten cluster or host block without ``k8s_distribution`` gets ``rke1`` -- the
   module default is RKE2, and a running RKE1 cluster cannot take RKE2 nodes;
4. after confirmation the previous document is kept as the blob
   ``main.tf.json.pre-migrate`` and the migrated one is persisted.

Nothing is applied: the next ``create`` (or an explicit re-apply) runs the new modules.
"""

import os
from typing import Any, Dict, List, Tuple

from ..backend.base import Backend
from ..config.context import Context
from ..errors import ConfigError, TKError
from ..models.common import source_for
from ..terraform import hcl
from ..terraform.catalog import local_module_dir, module_from_source
from ..terraform.plan import plan_module
from .create import NO_MANAGERS
from .select import select_manager

BACKUP_BLOB = "main.tf.json.pre-migrate"


def plan_migration(ctx: Context, doc: Dict[str, Any], drop_unknown: bool = False
                   ) -> Tuple[Dict[str, Dict[str, Any]], List[str], List[str]]:
    """``(new module blocks by key, errors, warnings)`` for a document's ``module`` map."""
    new_blocks: Dict[str, Dict[str, Any]] = {}
    errors: List[str] = []
    warnings: List[str] = []
    for key, block in (doc.get("module") or {}).items():
        if not isinstance(block, dict):
            errors.append(f"module.{key}: not a module block (an object)")
            continue
        src = str(block.get("source", ""))
        info = module_from_source(src)
        if info is None:
            errors.append(f"module.{key}: unknown module source {src!r}")
            continue
        target = source_for(ctx, info.path)
        if src == target:
            continue
        new = dict(block, source=target)
        mod_dir = local_module_dir(target) or info.local_dir
        if not os.path.isdir(mod_dir):
            errors.append(f"module.{key}: the module directory of {target!r} ({mod_dir}) does not exist here")
            continue
        if "k8s_distribution" not in new and "k8s_distribution" in hcl.check_module(mod_dir).variables:
            new["k8s_distribution"] = "rke1"
            warnings.append(f"module.{key}: k8s_distribution set to rke1 (the reference's clusters are RKE1)")
        problems = hcl.check_inputs(mod_dir, new)
        for p in problems:
            if p.startswith("unsupported argument "):
                arg = p.split("'")[1]
                if drop_unknown:
                    new.pop(arg, None)
                    warnings.append(f"module.{key}: dropped {arg!r} (not a variable of {info.name})")
                else:
                    errors.append(f"module.{key}: {p} of {info.name} (set migrate_drop_unknown: true to drop it)")
            elif p.startswith("missing required argument "):
                errors.append(f"module.{key}: {p} of {info.name}")
            else:
                warnings.append(f"module.{key}: {p} (terraform plan refuses this until it is changed)")
        if not any(e.startswith(f"module.{key}:") for e in errors):
            # every expression of the new module for these inputs (terraform/plan.py)
            for p in plan_module(mod_dir, new, check_files=False).errors:
                if "Invalid value for variable" not in p:  # check_inputs reported it above
                    warnings.append(f"module.{key}: plan: {p}")
        new_blocks[key] = new
    return new_blocks, errors, warnings


def migrate_manager(ctx: Context, backend: Backend) -> None:
    managers = backend.states()
    if not managers:
        raise ConfigError(NO_MANAGERS)
    manager = select_manager(ctx, managers)
    state = backend.state(manager)
    drop = ctx.settings.get_bool("migrate_drop_unknown") if ctx.is_set("migrate_drop_unknown") else False
    new_blocks, errors, warnings = plan_migration(ctx, state.doc, drop)
    for key in sorted(new_blocks):
        ctx.echo(f"module.{key}: {state.module(key).get('source')} -> {new_blocks[key]['source']}")
    for w in warnings:
        ctx.echo(f"warning: {w}")
    if errors:
        raise TKError("migration refused:\n  " + "\n  ".join(errors))
    if not new_blocks:
        ctx.echo(f'Cluster manager "{manager}" already uses this framework\'s modules.')
        return
    if not ctx.confirm(f'Migrate "{manager}" ({len(new_blocks)} modules)', f'Migrate "{manager}"'):
        ctx.echo("Migrate manager canceled.")
        return
    with backend.lock(manager):
        # the plan was made (and confirmed) on the document read before the lock: refuse
        # rather than overwrite what another CLI persisted in between
        if backend.state(manager).bytes() != state.bytes():
            raise TKError(f'Cluster manager "{manager}" changed while the migration was being confirmed; '
                          "run migrate again.")
        try:
            backend.write_blob(manager, BACKUP_BLOB, state.bytes())
        except NotImplementedError:
            pass
        for key, block in new_blocks.items():
            state.set_module(key, block)
        backend.persist_state(state)
    ctx.echo(f'Cluster manager "{manager}" migrated; the previous document is kept as {BACKUP_BLOB}.')


__all__ = ["migrate_manager", "plan_migration", "BACKUP_BLOB"]
