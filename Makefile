# Developer entry points (reference Makefile builds the docs site; this one drives the framework).
PY ?= python
ENV_DIR ?= .tt-env

.PHONY: build test test-gpu bench bench-query up down status validate what-if docs docs-local clean

build:            ## compile native (C++) engines and gfx950 HIP kernels in-tree
	$(PY) -c "import __graft_entry__ as g; g.build()"

test:             ## CPU test suite
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu:         ## GPU tests (MI355X)
	$(PY) -m pytest tests -q -m gpu

bench:            ## end-to-end createTask throughput (one JSON line)
	$(PY) bench.py

bench-query:      ## GPU state-query scan microbenchmark
	$(PY) bench_query.py

validate:
	$(PY) -m aca_dotnet_workshop_amd.platform validate -f deploy/main.yaml -p deploy/main.parameters.json

what-if:
	$(PY) -m aca_dotnet_workshop_amd.platform what-if -f deploy/main.yaml -p deploy/main.parameters.json --env-dir $(ENV_DIR)

up:               ## deploy the environment locally (detached)
	$(PY) -m aca_dotnet_workshop_amd.platform up -f deploy/main.yaml -p deploy/main.parameters.json --env-dir $(ENV_DIR) --detach

status:
	$(PY) -m aca_dotnet_workshop_amd.platform status --env-dir $(ENV_DIR)

down:
	$(PY) -m aca_dotnet_workshop_amd.platform down --env-dir $(ENV_DIR)

docs:             ## build the docs site (needs mkdocs-material)
	mkdocs build --strict

docs-local:
	mkdocs serve

clean:
	rm -rf $(ENV_DIR) build .pytest_cache
	find . -name __pycache__ -type d -prune -exec rm -rf {} +
