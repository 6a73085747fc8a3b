"""Re-run one setup of scripts/soak_consumer.py, twice with mOS's real clock and
twice frozen, and print what differs (diagnostic, not a test).

    python3 scripts/repro_soak_consumer.py [emul|gpu] [seed=7] [setup=3]
"""
import os, sys, random, tempfile, pathlib
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("scripts", "tests", "mos-networking-stack_amd"):
    sys.path.insert(0, os.path.join(ROOT, d))
import soak_consumer as S, test_mos_consumer as T, pktlib
exe = T.APP if len(sys.argv) > 1 and sys.argv[1] == "gpu" else T.APP_EMUL
rnd = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 7)
fixtures = {fix: T.fixture_frames(fix) for fix in ("edge", "rand_small", "rand_mid")}
for count in range((int(sys.argv[3]) if len(sys.argv) > 3 else 3) + 1):
    sc = S.setup(rnd)
    fr = pktlib.conversation_frames(sc["nflows"], seed=sc["seed"], listen_port=sc["listen"])
    if rnd.random() < 0.3:
        extra = [f for fix in ("edge", "rand_small", "rand_mid") for f in fixtures[fix]]
        for f in rnd.sample(extra, k=rnd.randint(1, 60)):
            fr.insert(rnd.randint(0, len(fr)), f)
print(sc, len(fr))
T.SCENARIOS["r"] = sc
for trial in range(4):
    sc["real_clock"] = trial < 2
    with tempfile.TemporaryDirectory() as td:
        tmp = pathlib.Path(td)
        pp = T.run_app(exe, "pp", tmp, "r", sc, fr)
        gpu = T.run_app(exe, "gpu", tmp, "r", sc, fr, sc.get("gpu_env"))
        print(trial, "returns", gpu["returns"] == pp["returns"], "state", gpu["state"] == pp["state"],
              "cb", gpu["callbacks"] == pp["callbacks"], "tx", gpu["tx"] == pp["tx"], len(gpu["tx"]), len(pp["tx"]), "real clock" if sc["real_clock"] else "frozen",
              "arp", sum(f[12:14] == b"\x08\x06" for f in gpu["tx"]), sum(f[12:14] == b"\x08\x06" for f in pp["tx"]))
        if gpu["tx"] != pp["tx"]:
            a, b = gpu["tx"], pp["tx"]
            for i, (x, y) in enumerate(zip(a, b)):
                if x != y:
                    print("first diff at", i, str(x)[:300], "|", str(y)[:300]); break
