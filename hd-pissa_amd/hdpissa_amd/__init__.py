"""hdpissa_amd -- MI355X-native HD-PiSSA per-step distributed orthogonal-adapter update.

Drop-in surface of the reference (hd_pissa.py):
  CustomLinearLayer, replace_with_custom_layer, get_parent_module, save_custom_model
  hd_pissa_step(model, lr, t, world_size, ...)   -- the optimizer-step block hp:352-398
  init_adam_states(model)                        -- hp:290-295
  lr_at / total_steps / warmup_steps_from        -- hp:302-307, 338-344
  HDPissaTrainer                                 -- the micro-step loop hp:316-351 around the step
  data.*                                         -- prompt / masking / collator / shard, hp:24-28, 158-277
  save_hdpissa_state / load_hdpissa_state        -- resume state (absent in the reference)
All arithmetic runs in libhdpissa.so (HIP, gfx950) -- see include/hdpissa.h.
"""
from .layer import (CustomLinearLayer, FactorArena, custom_layers, flush_probes, get_parent_module,
                    init_adam_states, replace_with_custom_layer)
from .schedule import lr_at, total_steps, warmup_steps_from
from .step import HDPissaStep, hd_pissa_step
from .checkpoint import export_merged_safetensors, load_hdpissa_state, save_custom_model, save_hdpissa_state
from .train import HDPissaTrainer
from . import data

__all__ = ["CustomLinearLayer", "FactorArena", "custom_layers", "get_parent_module", "init_adam_states",
           "replace_with_custom_layer", "flush_probes", "lr_at", "total_steps", "warmup_steps_from", "HDPissaStep",
           "hd_pissa_step", "save_custom_model", "export_merged_safetensors", "save_hdpissa_state",
           "load_hdpissa_state", "HDPissaTrainer", "data"]
