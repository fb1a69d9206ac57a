#!/bin/bash
# PCIe ceiling: tools/debug/pcie_probe with the runtime's default copy path,
# SDMA forced on, and SDMA off (blit kernels)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for v in default 1 0; do
  echo "== HSA_ENABLE_SDMA=$v"
  if [ $v = default ]; then timeout -k 10 120 tools/debug/pcie_probe || exit $?
  else HSA_ENABLE_SDMA=$v timeout -k 10 120 tools/debug/pcie_probe || exit $?; fi
done
