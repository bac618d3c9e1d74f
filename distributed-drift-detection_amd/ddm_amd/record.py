"""Post-loop record: DDM_Process.py:250-273 after the partition
function has run.

  * `dist_between_changes = num_rows // number_of_changes` (:53-55): rows of the prepared
    stream (after MULT) over the number of distinct targets;
  * `calc_change_dist(changes) = changes % dist_between_changes` (:250-254) on
    change_flag_global, then `df.where(change_flag_global != -1).dropna()` (:257): only the
    batches with a change survive, as float64 (the `where` masks to NaN first);
  * `total_time` from the partition dispatch to the collected frame (:224, :258);
  * one results row (APP_NAME, TIME_STRING, URL, INSTANCES, MULT, MEMORY, CORES,
    total_time, mean distance) appended to the rows read from `ddm_cluster_runs.csv` and
    written to `sparse_cluster_runs.csv` (:262-273; the reference reads one file and writes
    the other -- both names are parameters here).
"""
import numpy as np
import pandas as pd

RESULT_COLUMNS = ["Spark App", "Exp Start Time", "Spark Address", "Instances", "Data Multiplier", "Memory",
                  "Cores", "Final Time", "Average Distance"]


def dist_between_changes(num_rows, target):
    """DDM_Process.py:53-55."""
    return int(num_rows) // len(pd.unique(np.asarray(target)))


def change_distances(events, dist):
    """DDM_Process.py:250-257: the event frame with a `distance` column, restricted to the
    batches with a change (float64, as `where(...).dropna()` leaves them)."""
    df = events.copy()
    df["distance"] = (df["change_flag_global"].to_numpy().astype(np.int64) % int(dist)).astype(np.int32)
    return df.where(df["change_flag_global"] != -1).dropna()


def results_row(app_name, time_string, url, instances, mult, memory, cores, total_time, mean_distance):
    """The tuple DDM_Process.py:270 appends."""
    return (app_name, time_string, url, int(instances), float(mult), memory, int(cores), float(total_time),
            float(mean_distance))


def append_results(row, read_path="ddm_cluster_runs.csv", write_path="sparse_cluster_runs.csv"):
    """DDM_Process.py:262-273: previous rows (if the file reads) + this row -> write_path."""
    try:
        passed = pd.read_csv(read_path, index_col=0).values.tolist()
    except (FileNotFoundError, pd.errors.EmptyDataError):
        passed = []
    out = pd.DataFrame(passed + [row], columns=RESULT_COLUMNS)
    out.to_csv(write_path)
    return out
