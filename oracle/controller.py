"""Oracle partition controller (test infrastructure only — see oracle/__init__.py).

Restates the reference's grouped-map partition function `run_DDM_loop`
(DDM_Process.py:170-213) and its helpers `train_rf` (:98-105), `predict_rf`
(:110-128) and `run_DDM` (:135-159):

  1. 100-row batches, last one short (:182-184);
  2. batch 0 shuffled -> training batch (:187), one `permutation(len)` draw of the
     GLOBAL numpy MT19937 (pandas `sample(frac=1)` == `np.random.permutation`);
  3. for every later batch: shuffle (:190, one permutation draw), refit on the
     training batch if flagged (:194-196, `RandomForestClassifier(n_jobs=CORES)`
     with random_state=None -> 100 `randint(2**31-1)` draws of the same global
     RNG), predict -> 0/1 error (:199, :117), DDM with carried state (:202),
     record the (warning, change) pair mapped to (local label, global row number);
  4. on a change: the shuffled batch becomes the training batch, the DDM is
     dropped, refit flagged (:207-210);
  5. fewer than 2 batches -> `ValueError("No objects to concatenate")` (:212).

`run_partition` works on numpy arrays; `run_partition_frames` keeps the
reference's pandas per-batch frames and `iterrows` DDM so that its cost profile
matches the reference (it is the bench's `cpu_baseline`, kind "port").
"""
import numpy as np
import pandas as pd
from sklearn.ensemble import RandomForestClassifier

from .ddm import CHANGE_LEVEL, MIN_NUM_DDM_VALS, PER_BATCH, WARNING_LEVEL, OracleDDM, scan_batch


def _fit(X, y, n_jobs):
    rf = RandomForestClassifier(n_jobs=n_jobs)       # random_state=None: global RNG (:102)
    rf.fit(X, y)
    return rf


def run_partition(X, y, local_labels, global_labels, n_jobs=1, per_batch=PER_BATCH,
                  ddm_params=(MIN_NUM_DDM_VALS, WARNING_LEVEL, CHANGE_LEVEL), record=None):
    """Events int64 [n_batches-1, 4] for one partition; consumes np.random's global state."""
    n = len(y)
    starts = list(range(0, n, per_batch))
    if len(starts) < 2:
        raise ValueError("No objects to concatenate")
    y = np.asarray(y)

    def rows_of(b):
        lo = starts[b]
        return lo + np.random.permutation(min(n, lo + per_batch) - lo)

    train_rows = rows_of(0)
    ddm, rf, retrain = None, None, True
    out = np.empty((len(starts) - 1, 4), dtype=np.int64)
    for b in range(1, len(starts)):
        rows = rows_of(b)
        if retrain:
            rf = _fit(X[train_rows], y[train_rows], n_jobs)
            retrain = False
        err = (rf.predict(X[rows]) != y[rows]).astype(np.int64)
        if ddm is None:
            ddm = OracleDDM(*ddm_params)
        w, c = scan_batch(err, ddm)
        out[b - 1] = (local_labels[rows[w]] if w >= 0 else -1, global_labels[rows[w]] if w >= 0 else -1,
                      local_labels[rows[c]] if c >= 0 else -1, global_labels[rows[c]] if c >= 0 else -1)
        if record is not None:
            record.append((b, rows, err))
        if c >= 0:
            train_rows, ddm, retrain = rows, None, True
    return out


def run_partition_chunked(X, y, local_labels, global_labels, n_jobs=1, per_batch=PER_BATCH,
                          ddm_params=(MIN_NUM_DDM_VALS, WARNING_LEVEL, CHANGE_LEVEL), max_chunk=4096):
    """`run_partition` with the classifier called on many batches at once: the same events
    and the same global RNG consumption, fast enough for partitions of millions of rows.

    Between two refits nothing the reference draws depends on the rows, so the shuffles of
    the next K batches are drawn in order (DDM_Process.py:190; the pending refit's 100 draws
    right after the first of them, :194-196) and one `predict` covers their rows
    (predict_rf is row-wise, :110-128).  The DDM then runs batch by batch (:202); at a change
    in batch c (:207-210) the generator goes back to the state right after batch c+1's
    shuffle, which the reference draws before the refit on batch c.  K doubles from 16 while
    no change occurs (at most max_chunk) and restarts at 16 after one."""
    n = len(y)
    starts = list(range(0, n, per_batch))
    nb = len(starts)
    if nb < 2:
        raise ValueError("No objects to concatenate")
    y = np.asarray(y)

    def rows_of(b):
        lo = starts[b]
        return lo + np.random.permutation(min(n, lo + per_batch) - lo)

    train_rows = rows_of(0)
    ddm, rf, retrain = None, None, True
    out = np.empty((nb - 1, 4), dtype=np.int64)
    b, K = 1, 16
    pending = None            # batch b's rows, already drawn (the batch after a change)
    while b < nb:
        K = min(K, nb - b)
        rows_l, states = [], []
        for k in range(K):
            if k == 0 and pending is not None:
                rows = pending
            else:
                rows = rows_of(b + k)
            if k == 0 and retrain:
                rf = _fit(X[train_rows], y[train_rows], n_jobs)
                retrain = False
            rows_l.append(rows)
            states.append(np.random.get_state())
        pending = None
        allrows = np.concatenate(rows_l)
        err_all = (rf.predict(X[allrows]) != y[allrows]).astype(np.int64)
        at, changed = 0, False
        for k in range(K):
            rows = rows_l[k]
            err = err_all[at:at + len(rows)]
            at += len(rows)
            if ddm is None:
                ddm = OracleDDM(*ddm_params)
            w, c = scan_batch(err, ddm)
            out[b + k - 1] = (local_labels[rows[w]] if w >= 0 else -1, global_labels[rows[w]] if w >= 0 else -1,
                              local_labels[rows[c]] if c >= 0 else -1, global_labels[rows[c]] if c >= 0 else -1)
            if c >= 0:
                train_rows, ddm, retrain = rows, None, True
                if k + 1 < K:                   # batch b+k+1 was drawn: keep it, undo the rest
                    np.random.set_state(states[k + 1])
                    pending = rows_l[k + 1]
                b += k + 1
                changed = True
                break
        if changed:
            K = 16
        else:
            b += K
            K = min(2 * K, max_chunk)
    return out


def run_partition_frames(pdf, x_features, n_jobs=1, per_batch=PER_BATCH):
    """Same semantics on pandas frames with the reference's per-batch frame building and
    `iterrows` DDM feed (its CPU cost profile).  Returns the reference's output frame."""
    if len(pdf) <= per_batch:
        raise ValueError("No objects to concatenate")
    chunks = [pdf.iloc[s:s + per_batch] for s in range(0, len(pdf), per_batch)]
    train = chunks[0].sample(frac=1)
    ddm, rf, retrain, rows = None, None, True, []
    for chunk in chunks[1:]:
        chunk = chunk.sample(frac=1)
        if retrain:
            rf = _fit(train[x_features].values, train["target"].values, n_jobs)
            retrain = False
        y = chunk["target"].values
        pred = rf.predict(chunk[x_features].values)
        res = pd.DataFrame({"y_true": y, "y_pred": pred, "accuracy": (pred != y).astype(int),
                            "full_df_row_number": chunk["full_df_row_number"]}, index=chunk.index)
        if ddm is None:
            ddm = OracleDDM()
        warn, chg = (-1, -1), (-1, -1)
        for label, r in res.iterrows():
            ddm.add(r["accuracy"])
            if ddm.in_warning_zone and warn == (-1, -1):
                warn = (label, r["full_df_row_number"])
            if ddm.in_concept_change:
                chg = (label, r["full_df_row_number"])
                break
        rows.append(pd.DataFrame({"warning_flag_local": warn[0], "warning_flag_global": warn[1],
                                  "change_flag_local": chg[0], "change_flag_global": chg[1]}, index=[0]))
        if chg[1] > -1:
            train, ddm, retrain = chunk, None, True
    return pd.concat(rows)
