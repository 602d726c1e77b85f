# This module has no outputs.
