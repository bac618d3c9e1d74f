"""Golden-fixture generator: runs the REFERENCE's own partition function here.

Runs only in the build container (it reads /root/reference, which does not exist
on the GPU box).  It compiles the reference's own function bodies straight from
`DDM_Process.py` and calls them; nothing of the reference is copied into the repo,
only the inputs and outputs below are committed.

  * lines 1-36   settings block             (DDM_Process.py:1-36)
  * lines 94-213 train_rf / predict_rf / run_DDM / run_DDM_loop (DDM_Process.py:94-213)

Two shims stand in for absent third-party modules:
  * `pyspark.sql.functions.pandas_udf` -> identity decorator (DDM_Process.py:164-169)
  * `skmultiflow.drift_detection.DDM`  -> restatement of scikit-multiflow 0.5.3
    `ddm.py` (the library is not installed anywhere here; its arithmetic is
    therefore "parity unpinned" against upstream).

Everything else is the real thing: pandas 2.3.3 `sample`, numpy's global
MT19937, scikit-learn 1.7.2 RandomForestClassifier fit/predict.

Data prep restates DDM_Process.py:42-51 with a seeded RNG and a STABLE sort (the
reference's quicksort is platform dependent, SURVEY.md finding 11); the resulting
row order is stored in the fixture so every consumer uses exactly this stream.
Partition seeding follows SURVEY.md §8c: `np.random.seed(base + device_id)`.

Outputs (tests/golden/):
  outdoor.npz           dataset as pandas parsed it (X f64 [4000,21], target i64)
  outdoor_cfg_*.npz     per (MULT, INSTANCES): order, per-partition events
  outdoor_trace.npz     per-batch error vectors, refit points, exported forests
                        and expected predictions for a few configs
  ddm_kat.npz           DDM known-answer p/s traces on crafted 0/1 sequences
  manifest.json         versions, seeds, configs, sha1 of each output frame

Usage:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys
import types

import numpy as np
import pandas as pd
import sklearn

REF = "/root/reference/DDM_Process.py"
CSV = "/root/reference/outdoorStream.csv"
HERE = os.path.dirname(os.path.abspath(__file__))

DATA_SEED = 123
BASE_SEED = 1000
CONFIGS = [(m, i) for m in (1, 2, 4) for i in (1, 2, 4, 8, 16)]
TRACE_CONFIGS = [(2, 1), (4, 16)]
TRACE_TREES = 3          # forests kept per partition (first fits only)
TRACE_TREE_PARTS = 4     # partitions whose forests are kept


# --------------------------------------------------------------------------- shims
class _DDMShim:
    """scikit-multiflow 0.5.3 DDM, restated (upstream source not available)."""

    def __init__(self, min_num_instances=30, warning_level=2.0, out_control_level=3.0):
        self.min_instances = min_num_instances
        self.warning_level = warning_level
        self.out_control_level = out_control_level
        self.reset()

    def reset(self):
        self.in_concept_change = False
        self.in_warning_zone = False
        self.estimation = 0.0
        self.delay = 0.0
        self.sample_count = 1
        self.miss_prob = 1.0
        self.miss_std = 0.0
        self.miss_prob_sd_min = float("inf")
        self.miss_prob_min = float("inf")
        self.miss_sd_min = float("inf")

    def add_element(self, prediction):
        if self.in_concept_change:
            self.reset()
        self.miss_prob = self.miss_prob + (prediction - self.miss_prob) / float(self.sample_count)
        self.miss_std = np.sqrt(self.miss_prob * (1 - self.miss_prob) / float(self.sample_count))
        self.sample_count += 1
        self.estimation = self.miss_prob
        self.in_concept_change = False
        self.in_warning_zone = False
        self.delay = 0
        if self.sample_count < self.min_instances:
            return
        if self.miss_prob + self.miss_std <= self.miss_prob_sd_min:
            self.miss_prob_min = self.miss_prob
            self.miss_sd_min = self.miss_std
            self.miss_prob_sd_min = self.miss_prob + self.miss_std
        if self.miss_prob + self.miss_std > self.miss_prob_min + self.out_control_level * self.miss_sd_min:
            self.in_concept_change = True
        elif self.miss_prob + self.miss_std > self.miss_prob_min + self.warning_level * self.miss_sd_min:
            self.in_warning_zone = True
        else:
            self.in_warning_zone = False

    def detected_warning_zone(self):
        return self.in_warning_zone

    def detected_change(self):
        return self.in_concept_change


def _install_shims():
    pyspark = types.ModuleType("pyspark")
    sql = types.ModuleType("pyspark.sql")
    funcs = types.ModuleType("pyspark.sql.functions")
    funcs.pandas_udf = lambda *a, **k: (lambda f: f)
    funcs.PandasUDFType = types.SimpleNamespace(GROUPED_MAP="GROUPED_MAP")
    funcs.col = funcs.when = funcs.udf = funcs.lit = None
    pyspark.sql = sql
    sql.functions = funcs
    skm = types.ModuleType("skmultiflow")
    dd = types.ModuleType("skmultiflow.drift_detection")
    dd.DDM = _DDMShim
    skm.drift_detection = dd
    sys.modules.update({"pyspark": pyspark, "pyspark.sql": sql, "pyspark.sql.functions": funcs,
                        "skmultiflow": skm, "skmultiflow.drift_detection": dd})


def load_reference_namespace(n_features):
    """Compile DDM_Process.py:1-36 and :94-213 (the reference's own text)."""
    _install_shims()
    with open(REF) as f:
        lines = f.read().split("\n")
    ns = {"__name__": "ddm_reference"}
    exec(compile("\n".join(lines[0:36]), REF, "exec"), ns)           # lines 1-36
    ns["NUMBER_OF_FEATURES"] = n_features
    ns["X_features"] = [str(i) for i in range(n_features)]          # :33-34 for this file
    ns["CORES"] = "1"                                                # outputs independent of CORES
    ns["pd"], ns["np"] = pd, np
    body = "\n" * 93 + "\n".join(lines[93:213])                     # keep line numbers
    exec(compile(body, REF, "exec"), ns)                            # lines 94-213
    return ns


# --------------------------------------------------------------------------- data prep
def prep_stream(df, mult, data_seed):
    """DDM_Process.py:44-51 with a seeded RNG and a stable sort (order pinned)."""
    np.random.seed(data_seed)
    if float(mult) < 1:
        d = df.sample(frac=float(mult))
    else:
        d = pd.concat([df] * int(float(mult))).sample(frac=1)
    d = d.sort_values(by="target", kind="stable")
    return d.index.to_numpy()            # full_df_row_number order (DDM_Process.py:220)


def partitions(df, order, instances):
    """DDM_Process.py:220-226: device_id = full_df_row_number % INSTANCES, RangeIndex."""
    full = df.loc[order].copy()
    full["full_df_row_number"] = order
    full["device_id"] = (order % instances).astype(np.int32)
    out = []
    for d in range(instances):
        part = full[full["device_id"] == d].reset_index(drop=True)
        out.append((d, part))
    return out


def _sha1(a):
    return hashlib.sha1(np.ascontiguousarray(a).tobytes()).hexdigest()


def export_tree_arrays(rf):
    """Raw sklearn arrays of every tree (the product exporter consumes these)."""
    trees = []
    for e in rf.estimators_:
        t = e.tree_
        trees.append(dict(left=t.children_left.astype(np.int32), right=t.children_right.astype(np.int32),
                          feature=t.feature.astype(np.int32), threshold=t.threshold.astype(np.float64),
                          value=t.value[:, 0, :].astype(np.float64),
                          missing_left=np.asarray(t.missing_go_to_left, dtype=np.uint8)))
    return trees


def run_config(ns, df, mult, instances, trace=False):
    order = prep_stream(df, mult, DATA_SEED)
    parts = partitions(df, order, instances)
    events = {}
    traces = {}
    for d, part in parts:
        rec = {"fits": [], "preds": [], "ddm": []}
        if trace:
            orig_train, orig_pred = ns["train_rf"], ns["predict_rf"]

            def train_rf(df_a, _o=orig_train, _r=rec):
                rf = _o(df_a)
                _r["fits"].append(dict(rows=df_a.index.to_numpy(), trees=export_tree_arrays(rf),
                                       classes=rf.classes_.astype(np.int64)))
                return rf

            def predict_rf(df_b, rf, _o=orig_pred, _r=rec):
                res = _o(df_b, rf)
                _r["preds"].append(dict(rows=df_b.index.to_numpy(), y_pred=res["y_pred"].to_numpy(),
                                        err=res["accuracy"].to_numpy().astype(np.uint8),
                                        fit_id=len(_r["fits"]) - 1))
                return res

            ns["train_rf"], ns["predict_rf"] = train_rf, predict_rf
        np.random.seed(BASE_SEED + d)
        if len(part) <= 100:
            try:
                ns["run_DDM_loop"](part)
                raise AssertionError("reference was expected to raise for <=100 rows")
            except ValueError as e:
                events[d] = ("ValueError", str(e))
        else:
            out = ns["run_DDM_loop"](part)
            events[d] = out[["warning_flag_local", "warning_flag_global",
                             "change_flag_local", "change_flag_global"]].to_numpy().astype(np.int64)
        if trace:
            ns["train_rf"], ns["predict_rf"] = orig_train, orig_pred
            traces[d] = rec
    return order, events, traces


def ddm_kat():
    """Known-answer p/s traces from the DDM shim on crafted sequences (Appendix A)."""
    rs = np.random.RandomState(7)
    seqs = {
        "zeros_then_one": [0, 0, 0, 0, 1],
        "one_first": [1, 0, 0, 0, 0, 0],
        "all_ones": [1] * 50,
        "alternating": [0, 1] * 40,
        "second_is_error": [0, 1, 0, 0, 0, 0, 1],
        "bern_0.05": list(rs.binomial(1, 0.05, 400)),
        "bern_0.3": list(rs.binomial(1, 0.3, 400)),
        "bern_step": list(rs.binomial(1, 0.02, 300)) + list(rs.binomial(1, 0.4, 300)),
    }
    out = {}
    for name, seq in seqs.items():
        ddm = _DDMShim(3, 0.5, 1.5)
        p, s, w, c = [], [], [], []
        for x in seq:
            ddm.add_element(np.int64(x))
            p.append(ddm.miss_prob); s.append(ddm.miss_std)
            w.append(ddm.in_warning_zone); c.append(ddm.in_concept_change)
        out[name + "/x"] = np.array(seq, dtype=np.uint8)
        out[name + "/p"] = np.array(p, dtype=np.float64)
        out[name + "/s"] = np.array(s, dtype=np.float64)
        out[name + "/warn"] = np.array(w, dtype=np.uint8)
        out[name + "/change"] = np.array(c, dtype=np.uint8)
    return out


def main():
    df = pd.read_csv(CSV)
    n_feat = df.shape[1] - 1
    ns = load_reference_namespace(n_feat)
    np.savez_compressed(os.path.join(HERE, "outdoor.npz"),
                        X=df[[str(i) for i in range(n_feat)]].to_numpy(np.float64),
                        target=df["target"].to_numpy(np.int64))
    manifest = {"sklearn": sklearn.__version__, "numpy": np.__version__, "pandas": pd.__version__,
                "data_seed": DATA_SEED, "base_seed": BASE_SEED, "reference": "DDM_Process.py:1-36,94-213",
                "configs": {}}
    for mult, inst in CONFIGS:
        trace = (mult, inst) in TRACE_CONFIGS
        order, events, traces = run_config(ns, df, mult, inst, trace=trace)
        blob = {"order": order.astype(np.int32), "mult": mult, "instances": inst}
        info = {}
        for d, ev in events.items():
            if isinstance(ev, tuple):
                blob[f"raises/{d}"] = np.array(ev[1])
                info[d] = {"raises": ev[0]}
            else:
                blob[f"events/{d}"] = ev
                info[d] = {"rows": int(len(ev)), "drifts": int((ev[:, 3] > -1).sum()),
                           "warnings": int((ev[:, 1] > -1).sum()), "sha1": _sha1(ev)}
        np.savez_compressed(os.path.join(HERE, f"outdoor_cfg_m{mult}_i{inst}.npz"), **blob)
        manifest["configs"][f"m{mult}_i{inst}"] = info
        if trace:
            tb = {}
            for d, rec in traces.items():
                for k, fit in enumerate(rec["fits"]):
                    tb[f"{d}/fit{k}/rows"] = fit["rows"].astype(np.int32)
                    tb[f"{d}/fit{k}/classes"] = fit["classes"]
                    if k >= TRACE_TREES or d >= TRACE_TREE_PARTS:
                        continue
                    for t, tr in enumerate(fit["trees"]):
                        for key, arr in tr.items():
                            tb[f"{d}/fit{k}/tree{t}/{key}"] = arr
                for k, pr in enumerate(rec["preds"]):
                    tb[f"{d}/pred{k}/rows"] = pr["rows"].astype(np.int32)
                    tb[f"{d}/pred{k}/y_pred"] = pr["y_pred"].astype(np.int64)
                    tb[f"{d}/pred{k}/err"] = pr["err"]
                    tb[f"{d}/pred{k}/fit_id"] = np.int32(pr["fit_id"])
            np.savez_compressed(os.path.join(HERE, f"outdoor_trace_m{mult}_i{inst}.npz"), **tb)
        print(f"m{mult} i{inst}: {info}", flush=True)
    np.savez_compressed(os.path.join(HERE, "ddm_kat.npz"), **ddm_kat())
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
