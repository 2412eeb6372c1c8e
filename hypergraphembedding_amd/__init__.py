"""MI355X-native FOBE / HOBE hypergraph embedding.

Drop-in for the FOBE (HG2V_BOOLEAN) / HOBE (HG2V_ALG_DIST) hot path of
JSybrandt/HypergraphEmbedding: same registry keys, signatures and
``hypergraph.proto`` messages as the reference package ``__init__``
(hypergraph_embedding/__init__.py:8-42), with the work done by hand-written
gfx950 HIP kernels behind the C ABI of libhgx.so (include/hgx.h).

Importing the package does not touch the GPU; the first embedding call
creates the device context and raises if libhgx.so or a device is missing.
"""

from .proto import (EvaluationMetrics, ExperimentalResult, Hypergraph,
                    HypergraphEmbedding)
from .hypergraph_util import (AddNodeToEdge, CompressRange,
                              CreateRandomHyperGraph, FromSparseMatrix,
                              Incidence, IsEmpty, Relabel, RemoveEdge,
                              RemoveNode, RemoveNodeFromEdge, ToCscMatrix,
                              ToCsrMatrix, ToEdgeCsrMatrix)
from .algebraic_distance import EmbedAlgebraicDistance
from .hg2v_sample import (AlgebraicDistanceSamples, BooleanSamples,
                          SamplesToModelInput, SimilarityRecord,
                          WeightedJaccardSamples)
from .hg2v_weighting import (ComputeSpans, UniformWeight, WeightByAlgebraicSpan,
                             WeightByDistance, WeightByDistanceCluster,
                             WeightByNeighborhood, WeightBySameTypeDistance)
from .hg2v_model import (BooleanModel, KerasModelToEmbedding,
                         UnweightedFloatModel)
from .proto_native import (ShardedEmbedding, read_embedding, read_incidence,
                           save_embedding, write_embedding)
from .combine_embeddings_util import (CombineEmbeddingsViaConcatenation,
                                      CombineEmbeddingsViaNodeEdgeClassifier)
from .evaluation_util import (EXPERIMENT_OPTIONS, CalculateCommunityPredictionMetrics,
                              NodeEdgeEmbeddingPrediction, RemoveRandomConnections,
                              RunLinkPredictionExperiment, SampleMissingConnections)
from .embedding import (COMBINATION_OPTIONS, DEBUG_SUMMARY_OPTIONS,
                        EMBEDDING_OPTIONS, CombineEmbeddings, Embed,
                        EmbedHg2vAdjJaccard, EmbedHg2vAlgDist, EmbedHg2vBoolean,
                        EmbedHg2vNeighborhoodWeightedJaccard)

__all__ = [
    # proto
    "Hypergraph", "HypergraphEmbedding", "EvaluationMetrics",
    "ExperimentalResult",
    # embedding
    "Embed", "EMBEDDING_OPTIONS", "DEBUG_SUMMARY_OPTIONS",
    "COMBINATION_OPTIONS", "CombineEmbeddings", "EmbedHg2vBoolean",
    "EmbedHg2vAlgDist", "EmbedAlgebraicDistance", "EmbedHg2vAdjJaccard",
    "EmbedHg2vNeighborhoodWeightedJaccard", "WeightedJaccardSamples",
    # hot-path pieces
    "BooleanSamples", "AlgebraicDistanceSamples", "SamplesToModelInput",
    "SimilarityRecord", "UniformWeight", "WeightByNeighborhood",
    "WeightByDistance", "WeightBySameTypeDistance", "WeightByDistanceCluster",
    "WeightByAlgebraicSpan", "ComputeSpans",
    "BooleanModel", "UnweightedFloatModel", "KerasModelToEmbedding",
    # hypergraph util
    "AddNodeToEdge", "RemoveNodeFromEdge", "RemoveNode", "RemoveEdge",
    "CreateRandomHyperGraph", "FromSparseMatrix", "IsEmpty", "ToCsrMatrix",
    "ToEdgeCsrMatrix", "ToCscMatrix", "Relabel", "CompressRange", "Incidence",
    # native proto I/O
    "read_incidence", "write_embedding", "read_embedding", "save_embedding",
    "ShardedEmbedding",
    # combiners and link-prediction evaluation
    "CombineEmbeddingsViaConcatenation",
    "CombineEmbeddingsViaNodeEdgeClassifier", "EXPERIMENT_OPTIONS",
    "CalculateCommunityPredictionMetrics", "NodeEdgeEmbeddingPrediction",
    "RemoveRandomConnections", "RunLinkPredictionExperiment",
    "SampleMissingConnections",
]
