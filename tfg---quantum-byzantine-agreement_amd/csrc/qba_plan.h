// qba_plan.h -- host-only planning of a resource compile (no device code):
// gate validation and the classical permutation mask, union-find registers,
// factor merge + Vose alias tables, the closed-form classification and the
// permutation stage tables, and the program image uploaded to the device.
// Split out of qba_resource.hip so the host logic builds and runs on its own
// under AddressSanitizer / UBSan (tools/sanitize, tests/test_sanitizers.py).
#pragma once

#include <stdint.h>

#include <vector>

#include "qba_internal.h"

struct HostFactor {
  std::vector<uint64_t> pat;  // outcome patterns (size K), bit N-1-q = qubit q
  std::vector<double> prob;
};

// 1. validate the gate triples; for the Q circuit remove the X gates that
//    commute to a classical output mask and check that mask is the layout
//    field g = pi(g) (tfg.py:33-37).  `kept` = the quantum gates.
int qba_plan_gates(int n, int kind, const int32_t *gates, int ngates, const int32_t *perm,
                   std::vector<int32_t> &kept);
// 2. entangled registers (union-find over the 2-qubit gates), each in
//    ascending qubit order, registers by ascending smallest qubit.
std::vector<std::vector<int>> qba_plan_registers(int N, const std::vector<int32_t> &gates);
// 4. merge factors (product support <= 256) and build the alias tables.
int qba_plan_program(int n, const std::vector<HostFactor> &facs, QbaHostProgram &hp);
// 5. host image of a compiled (not-Q, Q) pair: QbaProgramSet + tables (+ the
//    closed form's stage tables).
int qba_plan_image(int n, const QbaHostProgram &a, const QbaHostProgram &b, std::vector<char> &img);
