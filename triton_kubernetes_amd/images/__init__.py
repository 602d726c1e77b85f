"""Machine-image templates (reference ``packer/``)."""

from .packer import TEMPLATES_DIR, load_template, render_template

__all__ = ["TEMPLATES_DIR", "load_template", "render_template"]
