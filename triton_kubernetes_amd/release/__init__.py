"""Release artefacts: single-file CLI, ``.deb``/``.rpm`` packages, checksums (reference ``Makefile``)."""
