"""Enterprise components (reference ``ee/``): PII redaction + consent
classification, envelope encryption, privacy API (consent / opt-out / DSAR
erasure fan-out / audit), policy broker (CEL tool policies), arena load tester,
eval worker.  Gated at runtime by the ``enterprise`` flag, as in the reference."""
