#!/bin/bash
# the host-side probes, built here in the container (tools/debug): PCIe
# ceiling, host DRAM bandwidth beside the DMA, CLI start-up pieces
# usage: tools/gpu/probes.sh TAG [pcie] [host_bw] [startup]
. "$(dirname "$0")/common.sh"
TAG=${1:-run}; shift
for p in ${*:-pcie host_bw startup}; do
    case $p in
    pcie) timeout -k 10 200 tools/debug/pcie_probe > $O/pcie_probe_$TAG.jsonl 2>&1 || { echo "pcie failed"; exit 1; } ;;
    host_bw) timeout -k 10 300 tools/debug/host_bw_probe ${HOST_BW_ARGS:-1024 4 16} > $O/host_bw_probe_$TAG.jsonl 2> $O/host_bw_probe_$TAG.err \
                 || { echo "host_bw failed"; tail $O/host_bw_probe_$TAG.err; exit 1; } ;;
    startup) for i in 1 2 3; do timeout -k 10 60 build/startup_probe >> $O/startup_probe_$TAG.jsonl 2>&1 || { echo "startup failed"; exit 1; }; done ;;
    esac
    echo "$p ok"; cat $O/*_probe_$TAG.jsonl | tail -12
done
