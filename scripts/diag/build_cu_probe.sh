#!/bin/bash
set -e
cd "$(dirname "$0")"
hipcc --offload-arch=gfx950 -O2 -fPIC -shared cu_probe.hip -o ../../boxfusion_amd/_build/cu_probe.so
