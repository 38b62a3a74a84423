"""``configs/parser.py:YAMLParser`` (defaults ``:32-66``, device ``:83-86``, seeds ``:92-96``,
``combine_entries`` ``:117-127``) -- the train_SNN.yml surface."""
import numpy as np
import torch
import yaml


class YAMLParser:
    def __init__(self, config):
        self.reset_config()
        self.parse_config(config)
        self.get_device()
        self.init_seeds()

    def parse_config(self, file):
        with open(file) as fid:
            self.parse_dict(yaml.safe_load(fid))

    @property
    def config(self):
        return self._config

    @property
    def device(self):
        return self._device

    @property
    def loader_kwargs(self):
        return self._loader_kwargs

    def reset_config(self):
        self._config = {
            "experiment": "Default",
            "data": {"mode": "events", "window": 5000},
            "loader": {"resolution": [180, 240], "batch_size": 1, "augment": [], "gpu": 0, "seed": 0},
            "hot_filter": {"enabled": True, "max_px": 100, "min_obvs": 5, "max_rate": 0.8},
            "model": {},
            "spiking_neuron": {},
            "vis": {"bars": False},
        }

    def update(self, config):
        self.reset_config()
        self.parse_config(config)

    def parse_dict(self, input_dict, parent=None):
        parent = self._config if parent is None else parent
        for key, val in input_dict.items():
            if isinstance(val, dict):
                parent.setdefault(key, {})
                self.parse_dict(val, parent[key])
            else:
                parent[key] = val

    def get_device(self):
        cuda = torch.cuda.is_available()
        self._device = torch.device("cuda:" + str(self._config["loader"]["gpu"]) if cuda else "cpu")
        self._loader_kwargs = {"num_workers": 0, "pin_memory": True} if cuda else {}

    @staticmethod
    def worker_init_fn(worker_id):
        np.random.seed(np.random.get_state()[1][0] + worker_id)

    def init_seeds(self):
        torch.manual_seed(self._config["loader"]["seed"])
        if torch.cuda.is_available():
            torch.cuda.manual_seed_all(self._config["loader"]["seed"])

    @staticmethod
    def combine_entries(config):
        if "spiking_neuron" in config.keys():
            config["model"]["spiking_neuron"] = config["spiking_neuron"]
            config.pop("spiking_neuron", None)
        return config


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
