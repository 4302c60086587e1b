# Build / run recipes (the reference's Makefile targets, /root/reference/Makefile:1-39,
# re-pointed at this framework: same role targets, plus the native build and tests).
PY ?= python
WORLD ?= 3
NPROC ?= 8
MASTER_PORT ?= 29500

.PHONY: build install setup graph first second server single gpu launch launch-gpu bench \
	bench-scale bench-scale-central test test-gpu profile dist clean asan

# compile every gfx950 HIP kernel + bindings into distributed_ml_pytorch_amd/_native*.so
build:
	$(PY) -m distributed_ml_pytorch_amd._build

install: build
	$(PY) -m pip install --no-build-isolation --no-deps -e .

# (reference: virtualenv + requirements); here the ROCm image already carries torch
setup: build

graph:
	mkdir -p docs
	$(PY) example/graph.py log docs

# three-process reference topology on one node: rank 0 = PS, ranks 1, 2 = workers
first:
	$(PY) example/main.py --rank 1 --world-size $(WORLD)

second:
	$(PY) example/main.py --rank 2 --world-size $(WORLD)

server:
	$(PY) example/main.py --rank 0 --world-size $(WORLD) --server

single:
	$(PY) example/main.py --no-distributed

gpu:
	$(PY) example/main.py --no-distributed --cuda

# all roles at once (replaces the AzureML submit of run-pytorch.py)
launch:
	$(PY) run-pytorch.py --nproc $(WORLD) -- --model lenet

launch-gpu:
	$(PY) run-pytorch.py --nproc $(NPROC) --gpus -- --cuda --model resnet18 --ps sharded

bench:
	$(PY) bench.py

bench-scale:
	for n in 1 2 4 8; do \
	  $(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $$n --master-addr 127.0.0.1 \
	    --master-port $(MASTER_PORT) bench.py --gpus $$n || exit $$?; \
	done

# the reference topology at every N: rank 0 = parameter server, ranks 1..N-1 = workers
# (BASELINE config #3 "1 PS + 7 workers"), payloads over one RCCL communicator per pair
bench-scale-central:
	for n in 2 4 8; do \
	  $(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $$n --master-addr 127.0.0.1 \
	    --master-port $(MASTER_PORT) bench.py --gpus $$n --ps central || exit $$?; \
	done

test:
	$(PY) -m pytest tests -x -q -m "not gpu"

# Host-side C++ under AddressSanitizer + UndefinedBehaviorSanitizer:
# every .hip file compiled HOST-ONLY (no device code, nothing is launched, no GPU
# needed) plus csrc/host_check.cpp, which drives the shape -> kernel-geometry
# logic and the 32-bit offset guards over every model's shapes and the oversize
# rejection paths.  The host-only objects each reference their (absent) fat
# binary: a generated stub defines those symbols.  Runs on the CPU.
ASAN_DIR ?= build/asan
CSRC := distributed_ml_pytorch_amd/csrc
HIPCC ?= /opt/rocm/bin/hipcc
ASAN_FLAGS := -O1 -g -std=c++17 -fno-omit-frame-pointer -I$(CSRC) \
	-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	-Xarch_host -fno-sanitize-recover=all
asan:
	mkdir -p $(ASAN_DIR)
	set -e; for f in $(CSRC)/*.hip; do \
	  $(HIPCC) -x hip --cuda-host-only $(ASAN_FLAGS) -c $$f -o $(ASAN_DIR)/$$(basename $$f .hip).o & \
	done; wait
	$(HIPCC) $(ASAN_FLAGS) -c $(CSRC)/host_check.cpp -o $(ASAN_DIR)/host_check.o
	nm $(ASAN_DIR)/*.o | awk '$$1 == "U" && $$2 ~ /^__hip_fatbin/ {print $$2}' | sort -u | \
	  awk '{printf "extern \"C\" __attribute__((aligned(4096))) const char %s[4096] = {0};\n", $$1}' \
	  > $(ASAN_DIR)/fatbin_stub.cpp
	g++ -c $(ASAN_DIR)/fatbin_stub.cpp -o $(ASAN_DIR)/fatbin_stub.o
	$(HIPCC) -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
	  $(ASAN_DIR)/*.o -o $(ASAN_DIR)/host_check
	ASAN_OPTIONS=detect_leaks=1 $(ASAN_DIR)/host_check

test-gpu:
	$(PY) -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread

profile:
	bash scripts/gpu_profile.sh

dist:
	$(PY) -m pip wheel --no-build-isolation --no-deps -w dist .

clean:
	rm -rf build dist distributed_ml_pytorch_amd/_native*.so
