"""MI355X-native FER-ViT models: drop-in for the reference's `models_fer_vit` package
(same constructors, attributes and state_dict keys; forward/backward run libfervit)."""
