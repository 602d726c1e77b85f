"""``python -m triton_kubernetes_amd`` == ``triton-kubernetes`` (reference ``main.go:5-7``)."""

import sys

from .cli.main import main

if __name__ == "__main__":
    sys.exit(main())
