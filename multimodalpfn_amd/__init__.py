"""MI355X-native drop-in for MultiModalPFN's inference hot path.

``from multimodalpfn_amd import MMPFNClassifier`` replaces
``from mmpfn.models.mmpfn import MMPFNClassifier``; ``ModelInterfaceConfig`` and
``PreprocessorConfig`` live in ``multimodalpfn_amd.constants`` /
``multimodalpfn_amd.preprocessing`` like their reference counterparts.
"""

__all__ = ["MMPFNClassifier"]


def __getattr__(name):
    if name == "MMPFNClassifier":
        from multimodalpfn_amd.classifier import MMPFNClassifier

        return MMPFNClassifier
    raise AttributeError(name)
