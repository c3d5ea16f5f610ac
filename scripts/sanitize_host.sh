#!/bin/bash
# AddressSanitizer + UBSan over the native HOST code (engine, data plane,
# schedule, simulator, bindings), driven by the CPU test suites.  Device code
# is not instrumented (GPU sanitizers are not available on this pool).
set -eo pipefail
cd "$(dirname "$0")/.."
SO=$(python -m akka_allreduce_amd._build --sanitize=address,undefined | tail -1)
ASAN_LIB=$(gcc -print-file-name=libasan.so)
UBSAN_LIB=$(gcc -print-file-name=libubsan.so)
export AKKA_NATIVE_PATH="$SO"
export ASAN_OPTIONS="detect_leaks=0:verify_asan_link_order=0:halt_on_error=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
# keep whatever is already preloaded, after the sanitizer runtimes
export LD_PRELOAD="$ASAN_LIB:$UBSAN_LIB${LD_PRELOAD:+:$LD_PRELOAD}"
python -m pytest -q -p no:cacheprovider tests/test_spec_worker.py tests/test_buffers.py tests/test_sim_schedule.py \
  tests/test_local_cluster.py tests/test_reactive_sim.py tests/test_faults.py tests/test_ipc_layout.py \
  tests/test_membership_epochs.py tests/test_racecheck.py tests/test_onesided_cpu.py tests/test_onesided_spec.py \
  -m "not gpu" "$@"
