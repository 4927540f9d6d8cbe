"""The build's scratch-memory gate (esmstereo_amd/build.py): every kernel's resource usage is parsed
from hipcc's kernel-resource-usage remarks, and a kernel outside ``SCRATCH_OK`` that uses scratch
memory fails the build.  CPU only: the parser on a sample of the remark text, and the reports the
last in-tree build left beside its objects."""
import glob
import json
import os

import pytest

from esmstereo_amd import build as B

SAMPLE = """\
x.hip:59:1: remark: Function Name: _ZN3esm4conv12_GLOBAL__N_112pair2_kernelILi5EEEv13esm_conv_descS3_ [-Rpass-analysis=kernel-resource-usage]
x.hip:59:1: remark:     TotalSGPRs: 40 [-Rpass-analysis=kernel-resource-usage]
x.hip:59:1: remark:     VGPRs: 108 [-Rpass-analysis=kernel-resource-usage]
x.hip:59:1: remark:     ScratchSize [bytes/lane]: 656 [-Rpass-analysis=kernel-resource-usage]
x.hip:80:1: remark: Function Name: _ZN3esm6other_kernelEv [-Rpass-analysis=kernel-resource-usage]
x.hip:80:1: remark:     VGPRs: 32 [-Rpass-analysis=kernel-resource-usage]
x.hip:80:1: remark:     ScratchSize [bytes/lane]: 0 [-Rpass-analysis=kernel-resource-usage]
"""


def test_kernel_resources_parser():
    res = B.kernel_resources(SAMPLE)
    assert res == {"_ZN3esm4conv12_GLOBAL__N_112pair2_kernelILi5EEEv13esm_conv_descS3_": {"vgpr": 108, "scratch": 656},
                   "_ZN3esm6other_kernelEv": {"vgpr": 32, "scratch": 0}}


def test_built_kernels_within_scratch_allowance():
    reports = sorted(glob.glob(os.path.join(B.BUILD, "*.o.res.json")))
    if not reports:
        pytest.skip("no in-tree build reports (build() not run in this tree)")
    n = 0
    for r in reports:
        with open(r) as f:
            res = json.load(f)
        n += len(res)
        for k, v in res.items():
            assert v.get("scratch", 0) <= B.SCRATCH_OK.get(k, 0), (os.path.basename(r), k, v)
    assert n > 100  # every source reported its kernels
