# Developer entry points (reference Makefile builds the docs site; this one drives the framework).
PY ?= python
ENV_DIR ?= .tt-env

.PHONY: build test test-gpu sanitize bench bench-query bench-query-e2e images up down status metrics validate what-if docs docs-local build-docs-website pipeline clean

build:            ## compile native engines, sidecar data plane, load generator and gfx950 HIP kernels in-tree
	$(PY) -c "import __graft_entry__ as g; g.build()"

test:             ## CPU test suite
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu:         ## GPU tests (MI355X)
	$(PY) -m pytest tests -q -m gpu

sanitize:         ## native engines + backing front under ThreadSanitizer and ASan/UBSan
	$(PY) -m pytest tests/test_native_sanitizers.py -q

bench:            ## end-to-end createTask throughput (one JSON line)
	$(PY) bench.py

bench-query:      ## GPU state-query scan microbenchmark (scan + ordering)
	$(PY) bench_query.py --sorted

bench-query-e2e:  ## state-query latency through the stack (GPU accelerator, 2M docs)
	$(PY) bench_query_e2e.py --docs 2000000 --accel gpu

images:           ## OCI images of the three services (standard + chiseled), verified under chroot when root
	$(PY) -m aca_dotnet_workshop_amd.platform image --out dist/images --verify

validate:
	$(PY) -m aca_dotnet_workshop_amd.platform validate -f deploy/main.yaml -p deploy/main.parameters.json

what-if:
	$(PY) -m aca_dotnet_workshop_amd.platform what-if -f deploy/main.yaml -p deploy/main.parameters.json --env-dir $(ENV_DIR)

up:               ## deploy the environment locally (detached)
	$(PY) -m aca_dotnet_workshop_amd.platform up -f deploy/main.yaml -p deploy/main.parameters.json --env-dir $(ENV_DIR) --detach

status:
	$(PY) -m aca_dotnet_workshop_amd.platform status --env-dir $(ENV_DIR)

metrics:          ## live metrics of the running environment
	$(PY) -m aca_dotnet_workshop_amd.platform metrics --env-dir $(ENV_DIR)

down:
	$(PY) -m aca_dotnet_workshop_amd.platform down --env-dir $(ENV_DIR)

SITE_DIR ?= dist/site

build-docs-website:  ## the workshop site, strict (reference Makefile target; used by the docs workflows)
	$(PY) -m aca_dotnet_workshop_amd.utils.docsite build --out $(SITE_DIR)

docs:             ## build the docs site with mkdocs-material instead (needs mkdocs)
	mkdocs build --strict

pipeline:         ## run a workflow locally: make pipeline FILE=.github/workflows/infra-deploy.yml ARGS="--var X=y"
	$(PY) -m aca_dotnet_workshop_amd.utils.pipeline $(FILE) $(ARGS)

docs-local:
	mkdocs serve

clean:
	rm -rf $(ENV_DIR) build .pytest_cache
	find . -name __pycache__ -type d -prune -exec rm -rf {} +
