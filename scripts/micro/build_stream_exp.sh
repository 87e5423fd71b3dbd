#!/bin/bash
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -shared -fPIC -o libstream_exp.so stream_exp.hip
