# triton-kubernetes (MI355X) build / test / release targets (reference Makefile).
VERSION    := v0.8.2
GIT_SHA    := $(shell git rev-parse --short HEAD 2>/dev/null || echo local)
PYTHON     ?= python3
BUILD      := build
PKG        := triton_kubernetes_amd

.PHONY: all native modules test test-gpu sanitize bench smoke dist pyz wheel build-deb build-rpm packages checksums clean

all: native test

# HIP/C++ probes for gfx950 (hipcc cross-compiles without a GPU)
native:
	PYTORCH_ROCM_ARCH=gfx950 $(PYTHON) -m $(PKG).ops.build -j 8

# regenerate terraform/modules from the generator (tests fail on drift)
modules:
	$(PYTHON) -m $(PKG).terraform.generate

test:
	$(PYTHON) -m pytest tests -x -q -m "not gpu"

# host-code memory/UB checks of the native labeller (ASan + UBSan build over a fixture tree)
sanitize:
	$(PYTHON) -m pytest tests/test_topology_native.py -q -k asan

# on an MI355X box
test-gpu: native
	$(PYTHON) -m pytest tests -x -q -m gpu

bench:
	$(PYTHON) bench.py --steps 10 --warmup 2

smoke:
	$(PYTHON) -c "import __graft_entry__ as g; g.build(); g.smoke()"

# single-file CLI (the reference ships one Go binary per OS); the git sha is
# injected like the reference's -ldflags -X cmd.cliVersion
pyz:
	rm -rf $(BUILD)/pyz && mkdir -p $(BUILD)/pyz
	cp -r $(PKG) $(BUILD)/pyz/
	find $(BUILD)/pyz -name __pycache__ -prune -exec rm -rf {} +
	rm -rf $(BUILD)/pyz/$(PKG)/ops/lib
	echo 'CLI_VERSION = "$(GIT_SHA)"' > $(BUILD)/pyz/$(PKG)/_build_info.py
	$(PYTHON) -m zipapp $(BUILD)/pyz -m "$(PKG).cli.main:main" -p "/usr/bin/env python3" \
		-o $(BUILD)/triton-kubernetes-$(VERSION).pyz

wheel:
	$(PYTHON) -m pip wheel --no-deps --no-build-isolation -w $(BUILD) .

# .deb / .rpm of the CLI and of the MI355X node tools, written with the stdlib
# (reference: fpm build-rpm / build-deb, Makefile:43-79); also writes sha256-checksums.txt
build-deb: native
	$(PYTHON) -m $(PKG).release.build --out $(BUILD) --formats pyz,deb

build-rpm: native
	$(PYTHON) -m $(PKG).release.build --out $(BUILD) --formats pyz,rpm

packages: native
	$(PYTHON) -m $(PKG).release.build --out $(BUILD) --formats pyz,deb,rpm

dist: packages

checksums:
	cd $(BUILD) && sha256sum triton-kubernetes-*.pyz *.deb *.rpm $$(ls *.whl 2>/dev/null) > sha256-checksums.txt

clean:
	rm -rf $(BUILD) $(PKG)/ops/lib
