"""Demo workloads: the RAG chat service (``rag_service``) whose spans the agent enriches,
backed by a stub generator or the random-init Llama model on an MI355X."""
