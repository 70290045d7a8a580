# Top-level build/test/image targets (reference: Makefile:16-65 build-<dist>/push-* targets).
VERSION ?= v0.1.0
IMAGE ?= amd-vgpu-device-plugin
PYTHON ?= python3

.PHONY: all native test test-gpu sanitize image bench suite scaling clean

all: native

native:
	$(MAKE) -C native -j8

test: native
	$(PYTHON) -m pytest tests -q -m "not gpu"

test-gpu: native
	$(PYTHON) -m pytest tests -q -m gpu

sanitize:
	$(MAKE) -C native -j8 SAN=thread
	$(MAKE) -C native -j8 SAN=address

image:
	docker build -f docker/Dockerfile --build-arg VERSION=$(VERSION) -t $(IMAGE):$(VERSION) .

bench: native
	$(PYTHON) bench.py

suite: native
	$(PYTHON) benchmarks/aibench_suite.py

scaling: native
	$(PYTHON) benchmarks/vgpu_scaling.py

clean:
	$(MAKE) -C native clean
