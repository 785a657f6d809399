#!/bin/bash
mkdir -p gpurun_out
for t in 256 1024; do
OI_SVGP_TIMING=1 OI_SVGP_THREADS=$t timeout -k 10 100 python -u -c "
import sys; sys.path.insert(0,'.')
import numpy as np
from oracle import svgp_oracle as O
from optimalinterpolation_amd import _lib
rng=np.random.default_rng(1); n=4600
x=np.stack([rng.uniform(-3e5,3e5,n),rng.uniform(-3e5,3e5,n),rng.integers(0,9,n).astype(float)],1); y=0.3+rng.normal(0,.02,n)
_lib.svgp_batch(x,y,[0,n],O.notebook_Z(x,50)[None],[[25e3,25e3,1,1,.1,.3]],[[0,0,4.]],batch=100,iterations=100)
" 2>&1 | grep phase
done
