#!/usr/bin/env bash
# Build the native runtime self-test with AddressSanitizer + UndefinedBehaviorSanitizer (host code only;
# GPU sanitizers are not used on this pool) and run it. usage: tools/sanitize_runtime.sh [seeds]
set -euo pipefail
here="$(cd "$(dirname "$0")/.." && pwd)"
rt="$here/generativeaiexamples_amd/csrc/runtime"
out="${TMPDIR:-/tmp}/gai_runtime_selftest_asan"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -I"$rt" "$rt/tests/runtime_selftest.cpp" "$rt/block_manager.cpp" "$rt/scheduler.cpp" -o "$out"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$out" "${1:-8}"
# constrained-decoding matcher: randomized walks under the same sanitizers
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=all \
    -I"$rt" "$rt/tests/grammar_selftest.cpp" "$rt/grammar.cpp" -o "${out}_grammar"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "${out}_grammar" "${1:-8}"
