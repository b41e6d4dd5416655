// Test stand-in for DBoW2::BowVector (Thirdparty/DBoW2/DBoW2/BowVector.h):
// word id -> weight, ascending (a std::map, as DBoW2's).
#pragma once
#include <map>

namespace DBoW2 {
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
class BowVector : public std::map<WordId, WordValue> {};
}  // namespace DBoW2
