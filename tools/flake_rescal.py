import sys, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "scikit-kge_amd"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tests"))
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import test_gpu_models as T
fails = 0
for i in range(int(sys.argv[1])):
    try:
        T.test_rescal_mfma_step_vs_oracle(400, 18, 200, 700)
    except AssertionError as e:
        fails += 1
        print("fail", i, str(e).splitlines()[0][:120])
print("fails", fails)
