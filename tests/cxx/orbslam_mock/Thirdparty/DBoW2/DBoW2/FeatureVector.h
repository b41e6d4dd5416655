// Test stand-in for DBoW2::FeatureVector (FeatureVector.h:20-23): node id ->
// feature indices, ascending node ids (a std::map, as DBoW2's).
#pragma once
#include <map>
#include <vector>

#include "BowVector.h"

namespace DBoW2 {
class FeatureVector : public std::map<NodeId, std::vector<unsigned int>> {};
}  // namespace DBoW2
