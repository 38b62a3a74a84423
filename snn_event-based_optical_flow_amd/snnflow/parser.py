"""The ``configs/train_SNN.yml`` model surface as ``train_flow.py`` hands it to a model.

The reference's own ``YAMLParser`` (``configs/parser.py:6-127``) is kept by the caller
(``train_flow.py`` keeps importing it); only the resulting ``unet_kwargs`` dict is restated here.
"""


def train_snn_model_kwargs(name="LIFFireNet", base_num_channels=8, num_bins=2, encoding="cnt", mask_output=True):
    """``unet_kwargs`` of the shipped training config: the ``model`` section of
    ``configs/train_SNN.yml:10-31`` with ``spiking_neuron`` moved under ``model``, as
    ``YAMLParser.combine_entries`` (``configs/parser.py:117-127``) hands it to the model."""
    return {
        "name": name, "encoding": encoding, "round_encoding": False, "norm_input": False,
        "num_bins": num_bins, "base_num_channels": base_num_channels, "kernel_size": 3,
        "activations": ["arctanspike", "arctanspike"], "mask_output": mask_output,
        "quantization": {"enabled": False, "PTQ": False, "Conv_only": False},
        "tebn": {"enabled": False, "num_timesteps": 4}, "mpbn": {"enabled": False},
        "spiking_neuron": {"leak": [0.0, 1.0], "thresh": [0.0, 0.8], "learn_leak": True,
                           "learn_thresh": True, "hard_reset": True},
    }
