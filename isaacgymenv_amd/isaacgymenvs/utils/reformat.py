"""``omegaconf_to_dict`` / ``print_dict`` (reference ``utils/reformat.py:32-58``).

The composer in ``isaacgymenvs/config.py`` already yields plain dicts; real
OmegaConf objects (if a user passes one) are converted through
``OmegaConf.to_container``."""


def omegaconf_to_dict(d):
    try:  # pragma: no cover - omegaconf is not installed in this image
        from omegaconf import DictConfig, OmegaConf
        if isinstance(d, DictConfig):
            return OmegaConf.to_container(d, resolve=True)
    except Exception:
        pass
    if isinstance(d, dict):
        return {k: omegaconf_to_dict(v) for k, v in d.items()}
    return d


def print_dict(val, nesting: int = -4, start: bool = True):
    if isinstance(val, dict):
        if not start:
            print("")
        nesting += 4
        for k in val:
            print(nesting * " ", end="")
            print(k, end=": ")
            print_dict(val[k], nesting, start=False)
    else:
        print(val)
