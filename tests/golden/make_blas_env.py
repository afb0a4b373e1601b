"""Records the numpy / OpenBLAS build the RANSAC and plane golden files were made with
(tests/golden/plane_digests.npz, ransac.json). The device restates numpy's LAPACK dgesv + dot, gemv and
pairwise-mean rounding of THIS build; tests/test_ransac_cpu.py checks that the numpy it
runs against is the same build, so a different numpy/OpenBLAS fails there by name instead of as a last-bit
plane mismatch. Run in the container: python tests/golden/make_blas_env.py"""
import json
import os

import numpy as np
import threadpoolctl


def env():
    blas = np.show_config(mode="dicts")["Build Dependencies"]["blas"]
    rt = [d for d in threadpoolctl.threadpool_info() if d.get("internal_api") == "openblas"]
    return {"numpy": np.__version__, "blas_name": blas.get("name"), "blas_version": blas.get("version"),
            "openblas_configuration": blas.get("openblas configuration"),
            "runtime_architecture": rt[0].get("architecture") if rt else None}


if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "blas_env.json")
    with open(out, "w") as fh:
        json.dump(env(), fh, indent=1)
        fh.write("\n")
    print(out, env())
