# llm-slo-ebpf-toolkit (MI355X-native). Targets mirror the reference workflow; every
# tool is `python -m llm_slo_ebpf_toolkit_amd.cli.<tool>` (bin/<tool> launchers).
PY ?= python3
CLI := $(PY) -m llm_slo_ebpf_toolkit_amd.cli
ART := artifacts

build:            ## compile HIP kernels (gfx950), native runtime, rocprofiler tool
	$(PY) -m llm_slo_ebpf_toolkit_amd.ops.build

test:             ## CPU test suite (no GPU needed)
	$(PY) -m pytest tests -q -m "not gpu"

test-gpu:         ## GPU tests (MI355X)
	$(PY) -m pytest tests -q -m gpu

RT := llm_slo_ebpf_toolkit_amd/runtime/csrc
RT_STRESS := tests/native/ring_stress.cpp $(RT)/ring.cpp $(RT)/bpfring.cpp $(RT)/pool.cpp

sanitize-asan:    ## host ring code under AddressSanitizer + UBSan (multi-producer stress)
	@mkdir -p build
	g++ -std=c++17 -O1 -g -pthread -fsanitize=address,undefined -fno-omit-frame-pointer -I$(RT) $(RT_STRESS) \
	    -o build/ring_stress_asan -lrt
	build/ring_stress_asan

sanitize-tsan:    ## host ring code under ThreadSanitizer (multi-producer stress)
	@mkdir -p build
	g++ -std=c++17 -O1 -g -pthread -fsanitize=thread -I$(RT) $(RT_STRESS) -o build/ring_stress_tsan -lrt
	build/ring_stress_tsan

lint:
	$(PY) -m compileall -q llm_slo_ebpf_toolkit_amd tests tools

schema-validate:
	$(CLI).schemavalidate

schema-export:
	$(CLI).sloctl schema export --root .

prereq-check:
	$(CLI).sloctl prereq check

kind-up:
	deploy/kind/kind-up.sh

kind-down:
	deploy/kind/kind-down.sh

observability-up:
	kubectl apply -k deploy/observability

observability-down:
	kubectl delete -k deploy/observability

rag-service:      ## demo RAG service (stub backend; LLM_BACKEND=llama for the MI355X model)
	$(PY) -m llm_slo_ebpf_toolkit_amd.demo.rag_service --backend $${LLM_BACKEND:-stub}

ebpf-gen:         ## BPF objects (needs clang -target bpf, libbpf headers, bpftool)
	$(MAKE) -C llm_slo_ebpf_toolkit_amd/probes/ebpf

ebpf-smoke:
	scripts/ebpf-smoke.sh

bench:            ## headline benchmark (one MI355X)
	$(PY) bench.py

bench-artifacts:  ## benchmark artefact bundle (REF benchgen)
	$(CLI).benchgen --out $(ART)/benchmarks --scenario mixed_faults

replay:
	$(CLI).faultreplay --scenario mixed --count 30 --with-signals --out $(ART)/fault-replay/fault_samples.jsonl

inject:
	$(CLI).faultinject --scenario mixed --count 24 --out $(ART)/fault-injection/raw_samples.jsonl

collector-smoke: inject
	$(CLI).collector --input $(ART)/fault-injection/raw_samples.jsonl --output jsonl \
	  --output-path $(ART)/collector/slo-events.jsonl

attribute: replay
	$(CLI).attributor --input $(ART)/fault-replay/fault_samples.jsonl --out $(ART)/attribution/attributions.jsonl \
	  --summary-out $(ART)/attribution/summary.json --confusion-out $(ART)/attribution/confusion.csv

correlation-gate:
	$(CLI).correlationeval --out $(ART)/correlation/eval_summary.json --predictions-out $(ART)/correlation/predictions.csv

incident-lab:     ## run every incident-lab scenario through the engine
	$(CLI).sloctl lab run --out $(ART)/incident-lab/report.json

chaos-matrix:
	scripts/chaos/run_fault_matrix.sh

m5-gate:
	$(CLI).m5gate --candidate-root $(ART)/weekly-benchmark --baseline-root $(ART)/weekly-benchmark/baseline

dashboards:
	$(PY) tools/gen_dashboards.py

.PHONY: build test test-gpu lint schema-validate schema-export prereq-check kind-up kind-down observability-up \
        observability-down rag-service ebpf-gen ebpf-smoke bench bench-artifacts replay inject collector-smoke \
        attribute correlation-gate incident-lab chaos-matrix m5-gate dashboards
