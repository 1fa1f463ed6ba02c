"""Shared constants (role of ``tcb/constants.py:7-49``)."""

from enum import Enum

# Accuracy results with this prefix are passed unreduced to Model.postprocess.
UNREDUCED_ACCURACY_OP_PREFIX = "tensor:"
# Eval results with this prefix are written to summaries.
SIMPLE_VALUE_RESULT_PREFIX = "simple_value:"


class BenchmarkMode(str, Enum):
    TRAIN = "training"
    EVAL = "evaluation"
    TRAIN_AND_EVAL = "training + evaluation"
    FORWARD_ONLY = "forward only"

    def __str__(self):  # printed as "BenchmarkMode.TRAIN" like the reference header
        return "BenchmarkMode.%s" % self.name


class NetworkTopology(str, Enum):
    """Device interconnect used by --hierarchical_copy.

    DGX1 / GCP_V100 are the reference's NVLink hybrid-cube matrices.  On a
    MI355X node every GPU has a direct xGMI link to every other GPU (7 links
    each), so XGMI_MESH groups are arbitrary and all pairs are peers.
    """
    DGX1 = "dgx1"
    GCP_V100 = "gcp_v100"
    XGMI_MESH = "xgmi_mesh"

    def __str__(self):
        return self.value


# Peer-access matrices (row i: which devices i can reach directly).
PEER_MATRIX = {
    NetworkTopology.DGX1: [
        "YYYYYNNN", "YYYYNYNN", "YYYYNNYN", "YYYYNNNY",
        "YNNNYYYY", "NYNNYYYY", "NNYNYYYY", "NNNYYYYY"],
    NetworkTopology.GCP_V100: [
        "YYYYNYNN", "YYYYNNNN", "YYYYNNNY", "YYYYNNNN",
        "NNNNYYYY", "YNNNYYYY", "NNNNYYYY", "NNYNYYYY"],
    NetworkTopology.XGMI_MESH: ["YYYYYYYY"] * 8,
}
