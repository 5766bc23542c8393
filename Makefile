# ome-amd developer targets (the CI workflow calls these).
PY ?= python
JOBS ?= 6
COVERAGE_MIN ?= 48

.PHONY: build lint test test-shard test-gpu coverage bench catalog crds deploy verify-generated clean

build:            ## compile every HIP extension for gfx950 + the native IO/runtime library
	$(PY) -c "import __graft_entry__ as g; g.build()"

lint:             ## syntax + import hygiene (ruff when available)
	$(PY) -m compileall -q ome_amd tests scripts bench.py __graft_entry__.py
	@if command -v ruff >/dev/null; then ruff check --select E9,F63,F7,F82 ome_amd tests; fi

test:             ## CPU suite (gloo for multi-process paths)
	$(PY) -m pytest tests/ -x -q -m "not gpu" -n $(JOBS)

SHARD ?= runtime
SHARD_control-plane = tests/test_controllers_cpu.py tests/test_policy_cpu.py tests/test_webhooks_cpu.py \
	tests/test_modelagent_cpu.py tests/test_kube_adapter_cpu.py tests/test_samples_cpu.py tests/test_e2e_cpu.py \
	tests/test_console_cpu.py
SHARD_storage = tests/test_objstore_cpu.py tests/test_hfhub_cpu.py tests/test_agents_cpu.py \
	tests/test_storage_modelconfig_cpu.py
SHARD_runtime = $(filter-out $(SHARD_control-plane) $(SHARD_storage),$(wildcard tests/test_*_cpu.py))
test-shard:
	$(PY) -m pytest -x -q -m "not gpu" -n $(JOBS) $(SHARD_$(SHARD))

test-gpu:         ## one MI355X: kernels vs fp32 references, engines, multi-process comm
	$(PY) -u -m pytest tests/ -x -v -m gpu --timeout 300 --timeout-method thread

coverage:
	$(PY) -m pytest tests/ -q -m "not gpu" -n $(JOBS) --cov=ome_amd --cov-report=term --cov-fail-under=$(COVERAGE_MIN)

bench:            ## headline: Llama-3-8B serving tokens/s on one GPU
	$(PY) bench.py

catalog:          ## regenerate runtimes, model catalog and samples
	$(PY) -m ome_amd.catalog --out config

crds:
	$(PY) -c "from ome_amd.api import schema; schema.write_all('config/crd')"

deploy:           ## regenerate the kustomize overlays (rbac, webhook, certmanager, model-agent, configmap, default)
	$(PY) -m ome_amd.deploy

verify-generated: catalog
	git diff --exit-code -- config/runtimes config/models config/samples
	$(PY) -m ome_amd.deploy --check

clean:
	rm -rf ome_amd/_lib/*.so build/
