# qmx — developer targets (the reference's `make run / run-prod / install / test / test-cov /
# clean`, for the MI355X framework).  PORT / CONFIG / GPUS override the defaults.
PORT ?= 8001
CONFIG ?= config.yaml
GPUS ?= 1
PY ?= python

.PHONY: build run run-prod run-python install test test-gpu test-cov bench bench-node api-reference clean

build:  ## hipcc --offload-arch=gfx950: the _qmx extension + C++ mock backends / load generator
	$(PY) -c "import __graft_entry__ as g; g.build()"

run: build  ## native data plane, rolling reload on config edits (quorum: uvicorn --reload)
	$(PY) -m quorum_amd.serve --impl native --config $(CONFIG) --port $(PORT) --gpus $(GPUS) --watch-config

run-prod: build
	$(PY) -m quorum_amd.serve --impl native --config $(CONFIG) --port 8000 --gpus $(GPUS)

run-python:  ## FastAPI / uvicorn front end, same semantics
	$(PY) -m quorum_amd.serve --impl python --config $(CONFIG) --port $(PORT)

install:
	$(PY) -m pip install -e . --no-build-isolation

test: build  ## CPU suite (no GPU needed)
	$(PY) -m pytest tests -m "not gpu" -q -n 4

test-gpu: build  ## MI355X suite
	$(PY) -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread

test-cov: build
	$(PY) -m pytest tests -m "not gpu" -q --cov=quorum_amd --cov-report=term-missing

bench: build  ## headline benchmark, 1 GPU
	$(PY) bench.py

bench-node: build  ## the node: bench.py launches its ranks itself
	$(PY) bench.py --gpus $(GPUS)

api-reference:  ## re-export api_reference/openapi.json from the conformance app
	$(PY) -c "import json; from quorum_amd.server.app import create_app; from quorum_amd.utils.config import load_config; \
	open('api_reference/openapi.json', 'w').write(json.dumps(create_app(lambda: load_config()).openapi(), indent=2, sort_keys=True) + '\n')"

clean:
	rm -rf .pytest_cache .hypothesis build dist *.egg-info htmlcov .coverage
	find . -type d -name __pycache__ -prune -exec rm -rf {} +
