"""Drop-in inference API (rvc_mlx.infer): RVC_MLX / PipelineMLX names backed by the MI355X engine."""
from .index import IndexIVFFlat, read_index
from .infer import RVC_MLX, RVCX, load_audio, load_voice_model, mlx_to_reference_state
from .models import CREPE, FCPE, HubertModel, PitchExtractor, RMVPE0Predictor, Synthesizer
from .pipeline import Config, PipelineMLX, PipelineRVCX, proposed_key

__all__ = ["RVC_MLX", "RVCX", "PipelineMLX", "PipelineRVCX", "Config", "HubertModel", "RMVPE0Predictor",
           "Synthesizer", "CREPE", "FCPE", "PitchExtractor", "load_audio", "load_voice_model", "mlx_to_reference_state", "proposed_key",
           "IndexIVFFlat", "read_index"]
