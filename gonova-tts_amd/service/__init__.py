"""Service counterpart of the reference's `services/tts` (WS protocol, queues, batcher)."""
