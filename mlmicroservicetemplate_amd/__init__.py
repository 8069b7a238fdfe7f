"""mlmicroservicetemplate_amd -- an MI355X-native ML model-serving microservice framework.

Capabilities of CodyRichter/MLMicroserviceTemplate (REST ``/``, ``/status``, ``/predict``,
async model init, orchestrator registration heartbeat, ``.env`` config, Docker layout),
re-designed MI355X-first: a dynamic micro-batcher feeding per-GPU engines that replay
hipGraphs of hand-written CDNA4 HIP kernels, with RCCL over xGMI for multi-replica and
tensor-parallel fan-out across the 8 GPUs of a node.
"""
__version__ = "0.1.0"
