"""Live roofline measurement of the dominant kernel of the bench step (filled per profile)."""


def measure(cfg, trainer, batch):
    return None
