"""profiles/<round>_valu_exo_step.json from one rocprofv3 --pmc pass of the
fp64 VALU counters over the env step kernel (tools/env_valu_pmc.sh).
usage: python tools/valu_summary.py ROUND CSV [ENVS_PER_LAUNCH]"""
import collections
import csv
import json
import os
import sys

import numpy as np


def main():
    rnd, path = sys.argv[1], sys.argv[2]
    envs = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if "exo_step" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    names = sorted({c for d in per.values() for c in d})
    med = {c: float(np.median([d[c] for d in per.values() if c in d])) for c in names}
    flops = (2 * med["SQ_INSTS_VALU_FMA_F64"] + med["SQ_INSTS_VALU_ADD_F64"] + med["SQ_INSTS_VALU_MUL_F64"]) * 64
    out = {"kernel": "exo_step_rp_kernel", "envs_per_launch": envs, "launches": len(per), "counters_median": med,
           "fp64_flops_per_launch": flops,
           "formula": "(2*SQ_INSTS_VALU_FMA_F64 + SQ_INSTS_VALU_ADD_F64 + SQ_INSTS_VALU_MUL_F64) * 64 (rocprofv3's "
                      "FLOPS expression for f64 VALU; issued wave instructions x 64 lanes, exec-mask agnostic: an "
                      "upper bound on useful lane-flops); transcendental f64 ops not counted",
           "fp64_flops_per_env_step": flops / envs,
           "source": f"rocprofv3 --pmc pass on bench.py --mode env (tools/env_valu_pmc.sh), {path}"}
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
    json.dump(out, open(os.path.join(here, f"{rnd}_valu_exo_step.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
